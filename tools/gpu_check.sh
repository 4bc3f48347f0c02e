#!/bin/bash
# GPU-box check: parity tests, one bench line, one rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash / fault / timeout ends the script.
# Usage (from the repo root, via gpurun):  bash tools/gpu_check.sh [tag] [pytest-args...]
set -u
TAG=${1:-r01}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"

stop_if_fatal() {  # exit codes other than 0 (ok) and 1 (test failures) mean crash/fault/timeout
    local rc=$1 what=$2
    echo "[$what] rc=$rc"
    if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
        echo "[$what] fatal exit code, stopping"
        exit "$rc"
    fi
}

echo "== pytest -m gpu"
timeout -k 10 900 python -m pytest tests -m gpu -q -rf "$@" > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?
tail -25 "$OUT/pytest_gpu_$TAG.log"
stop_if_fatal $rc pytest

echo "== bench"
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?
cat "$OUT/bench_$TAG.json"; tail -5 "$OUT/bench_$TAG.err"
stop_if_fatal $rc bench
[ $rc -eq 0 ] || exit $rc

echo "== rocprofv3 kernel trace"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof_bench_$TAG.json" 2> "$OUT/prof_$TAG.err"
rc=$?
echo "[rocprofv3] rc=$rc"
tail -3 "$OUT/prof_$TAG.err"
find "$OUT/prof_$TAG" -name "*stats*" | head
[ $rc -eq 0 ] || exit $rc
if [ "${PMC:-0}" = "1" ]; then
    echo "== rocprofv3 pmc (SQ instruction mix)"
    timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
        --output-format csv -d "$OUT/prof_$TAG/pmc_sq1" -o run -- \
        python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> "$OUT/prof_${TAG}_pmc.err"
    rc=$?
    echo "[pmc] rc=$rc"
fi
exit $rc
