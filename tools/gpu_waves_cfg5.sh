#!/bin/bash
# A/B of the draw grid (CSA_DRAW_WAVES) for the general draw kernel at the synthetic n=8192 shape
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
for rep in 1 2; do
  for m in 1 0 2; do
    CSA_DRAW_WAVES=$m timeout -k 10 200 python bench.py --config synthetic8192 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/b_cfg5w.json" 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { echo "bench waves=$m rc=$rc"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels']; print('cfg5 waves %s %6.2fM/s draw alone %.3f ms (%s)' % (sys.argv[2], d['value']/1e6, k['draw']['ms'], k['draw']['kernel']))" "$OUT/b_cfg5w.json" $m
  done
done
