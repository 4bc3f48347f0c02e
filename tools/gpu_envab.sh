#!/bin/bash
# A/B of draw layouts by environment (CSA_DRAW_KERNEL=...) on one config's bench, after a pytest subset.
# Usage (repo root, via gpurun):  bash tools/gpu_envab.sh CONFIG "wide wide4" [pytest -k expr]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
CFG=$1; KS=$2; KEXPR=${3:-}
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$KEXPR" > "$OUT/pytest_envab.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest_envab.log"; echo "[pytest] rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
for rep in $(seq 1 "${REPS:-2}"); do
  for kk in $KS; do
    CSA_DRAW_KERNEL=$kk timeout -k 10 300 python bench.py --config "$CFG" --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-api \
        > "$OUT/envab_$kk.json" 2> "$OUT/envab.err"
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $kk"; tail -3 "$OUT/envab.err"; exit $rc; }
    python3 -c "
import json,sys; d=json.load(open('$OUT/envab_$kk.json')); k=d['kernels']; c=d['checks']
print('%-8s %8.2fM/s  draw %s %.3f / %.3f  pairs %.3f  checks %s' % (sys.argv[1], d['value']/1e6, k['draw'].get('kernel'), k['draw']['ms'],
      k['draw']['ms_in_timed_region'], k.get('pairs_mfma', {}).get('ms', 0),
      (c['last_step_unique'], c['last_step_count_sum'], c['last_step_pair_sum'])))" "$kk"
  done
done
