#!/bin/bash
# rocprofv3 passes for the LEGACY kernels (run on the GPU box from the repo root):
#   1. kernel trace + stats (csv)
#   2..n. one --pmc pass per counter group (never combined with trace domains)
# Usage: bash tools/gpu_prof.sh TAG [bench args...]
set -u
TAG=${1:-r01}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
BENCH=("$ROOT/bench.py" --steps 3 --warmup 1 --iso-steps 0 --no-cpu-baseline --no-api "$@")

run() {  # name, rocprofv3 args...
    local name=$1; shift
    timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- python3 "${BENCH[@]}" \
        > "$OUT/$name.json" 2> "$OUT/$name.err"
    local rc=$?
    echo "[$name] rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.err"; exit $rc; fi
}

run trace --kernel-trace --stats
if [ "${LIST_COUNTERS:-0}" = "1" ]; then
    timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
fi
run pmc_sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
run pmc_sq2 --pmc SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INST_LEVEL_LDS GRBM_GUI_ACTIVE
run pmc_fetch --pmc FETCH_SIZE
run pmc_write --pmc WRITE_SIZE
run pmc_mfma --pmc SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
echo done
