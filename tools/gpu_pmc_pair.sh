#!/bin/bash
# PMC passes over tools/pair_bench.py (one counter group per rocprofv3 run).
# Usage: bash tools/gpu_pmc_pair.sh TAG [pair_bench args...]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=${1:-pp}; shift || true
export TMPDIR=/tmp; cd /tmp
OUT=$ROOT/gpurun_out/prof_$TAG; mkdir -p "$OUT"
DEF="trace:--kernel-trace --stats|pmc_a:--pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU|pmc_b:--pmc SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE|pmc_fetch:--pmc FETCH_SIZE|pmc_write:--pmc WRITE_SIZE|pmc_tcc:--pmc TCC_HIT_sum TCC_MISS_sum"
IFS='|' read -ra PS <<< "${PASSES:-$DEF}"
for pass in "${PS[@]}"; do
  name=${pass%%:*}; args=${pass#*:}
  timeout -k 10 200 rocprofv3 $args -d "$OUT/$name" -o run --output-format csv -- python3 "$ROOT/tools/pair_bench.py" --reps 1 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/$name.err"; exit $rc; }
done
