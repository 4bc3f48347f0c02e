#!/bin/bash
# One GPU-box round trip: parity tests, the default bench line, rocprofv3 trace + PMC passes.
# Every GPU step has its own time limit; a crash / fault / timeout (exit code other than 0 / 1)
# ends the script.  Usage (repo root, via gpurun):  bash tools/gpu_round.sh TAG [pytest -k expr]
set -u
TAG=${1:-r02}
KEXPR=${2:-}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  if [ -n "$KEXPR" ]; then KARGS=(-k "$KEXPR"); else KARGS=(); fi
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 120 --timeout-method thread "${KARGS[@]}" \
      > "$OUT/pytest_$TAG.log" 2>&1
  rc=$?; tail -8 "$OUT/pytest_$TAG.log"; echo "[pytest] rc=$rc"
  fatal $rc && exit $rc
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
  rc=$?; cut -c1-1500 "$OUT/bench_$TAG.json"; tail -3 "$OUT/bench_$TAG.err"; echo "[bench] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${SKIP_PROF:-0}" != "1" ]; then
  bash tools/gpu_prof.sh "$TAG" ${PROF_ARGS:-}
  rc=$?; echo "[prof] rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
echo done
