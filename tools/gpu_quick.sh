#!/bin/bash
# GPU-box quick loop: parity tests (optionally filtered), then one bench line.
# Usage: bash tools/gpu_quick.sh TAG [pytest -k expr] [bench args...]
set -u
TAG=${1:-q}; shift || true; KEXPR=${1:-}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
if [ -n "$KEXPR" ]; then KARGS=(-k "$KEXPR"); else KARGS=(); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KARGS[@]}" > "$OUT/pytest_$TAG.log" 2>&1
rc=$?; tail -15 "$OUT/pytest_$TAG.log"; echo "[pytest] rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?; cat "$OUT/bench_$TAG.json"; tail -3 "$OUT/bench_$TAG.err"; echo "[bench] rc=$rc"
exit $rc
