#!/bin/bash
# bench the lane draw kernel's group sizes (CSA_DRAW_LANE=1|2|4), alternating
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
for rep in 1 2; do
  for g in 2 4 1; do
    CSA_DRAW_LANE=$g timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/b_lane$g.json" 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { echo "bench G=$g rc=$rc"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels']; print('G=%s %6.1fM/s draw %.3f ms (%s)' % (sys.argv[2], d['value']/1e6, k['draw']['ms'], k['draw']['kernel']))" "$OUT/b_lane$g.json" $g
  done
done
