#!/bin/bash
# PMC passes (SQ instruction mix / stalls / LDS) over the bench for each CSA_DRAW_GROUP.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=${1:-pd}; shift || true; GL=${1:-8 4}; shift || true
export TMPDIR=/tmp; cd /tmp
for g in $GL; do
  OUT=$ROOT/gpurun_out/prof_${TAG}_g$g; mkdir -p "$OUT"
  for pass in "trace:--kernel-trace --stats" \
              "pmc_sq1:--pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
              "pmc_sq2:--pmc SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INST_LEVEL_LDS GRBM_GUI_ACTIVE"; do
    name=${pass%%:*}; args=${pass#*:}
    CSA_DRAW_GROUP=$g timeout -k 10 300 rocprofv3 $args -d "$OUT/$name" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-pairs "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
    rc=$?; echo "[G=$g $name] rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/$name.err"; exit $rc; }
  done
done
