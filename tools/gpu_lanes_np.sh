#!/bin/bash
# A/B of the lane kernel group size (CSA_DRAW_LANE = 1 / 2 / 4) with the non-persistent launch
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
for rep in 1 2; do
  for g in 2 1 4; do
    CSA_DRAW_LANE=$g CSA_DRAW_WAVES=0 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/b_lnp.json" 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { echo "bench lane=$g rc=$rc"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels']; print('lane G=%s %6.1fM/s draw alone %.3f in-region %.3f (%s)' % (sys.argv[2], d['value']/1e6, k['draw']['ms'], k['draw']['ms_in_timed_region'], k['draw']['kernel']))" "$OUT/b_lnp.json" $g
  done
done
