#!/bin/bash
# A/B of the draw grid size (CSA_DRAW_WAVES: 1 = persistent, m = m resident grids, 0 = one workgroup
# per 128 panels) on the default bench workload, after the draw parity tests
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
for m in 1 2 0; do
  CSA_DRAW_WAVES=$m timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "draw or parity" > "$OUT/pytest_waves$m.log" 2>&1
  rc=$?; tail -1 "$OUT/pytest_waves$m.log"; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for m in 1 2 0; do
    CSA_DRAW_WAVES=$m timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/b_waves$m.json" 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { echo "bench waves=$m rc=$rc"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels']; print('waves %s %6.1fM/s ms/step %.3f draw alone %.3f in-region %.3f pairs-in-region %.3f' % (sys.argv[2], d['value']/1e6, d['ms_per_step'], k['draw']['ms'], k['draw']['ms_in_timed_region'], k['pairs_mfma']['ms_in_timed_region']))" "$OUT/b_waves$m.json" $m
  done
done
