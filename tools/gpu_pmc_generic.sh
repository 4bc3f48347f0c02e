#!/bin/bash
# PMC passes over bench.py (any bench args), one counter group per rocprofv3 run.
# Usage: bash tools/gpu_pmc_generic.sh TAG [bench args...]   (env PASSES overrides the default groups)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=${1:-pg}; shift || true
export TMPDIR=/tmp; cd /tmp
OUT=$ROOT/gpurun_out/prof_$TAG; mkdir -p "$OUT"
DEF="trace:--kernel-trace --stats|pmc_a:--pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU|pmc_b:--pmc SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
IFS='|' read -ra PS <<< "${PASSES:-$DEF}"
for pass in "${PS[@]}"; do
  name=${pass%%:*}; args=${pass#*:}
  timeout -k 10 300 rocprofv3 $args -d "$OUT/$name" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/$name.err"; exit $rc; }
done
