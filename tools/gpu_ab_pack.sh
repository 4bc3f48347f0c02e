#!/bin/bash
# A/B of the pick-list pack placement (draw stream vs counting stream) and pipeline depth.
set -u
cd ${GRAFT_REPO_ROOT:-.}; OUT=gpurun_out; mkdir -p $OUT
for rep in 1 2; do
  for cfg in "--pack-on draw --bufs 3" "--pack-on count --bufs 3" "--pack-on count --bufs 4" "--pack-on draw --bufs 4"; do
    timeout -k 10 200 python bench.py --steps 200 --warmup 3 --no-cpu-baseline --no-api $cfg > $OUT/ab.json 2> $OUT/ab.err
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $cfg"; tail -3 $OUT/ab.err; exit $rc; }
    python3 -c "import json,sys; d=json.load(open('$OUT/ab.json')); k=d['kernels']; print('%-26s %7.2fM/s  draw %.3f/%.3f pack %.3f/%.3f pairs %.3f' % (sys.argv[1], d['value']/1e6, k['draw']['ms'], k['draw']['ms_in_timed_region'], k['pack']['ms'], k['pack']['ms_in_timed_region'], k['pairs_mfma']['ms_in_timed_region']))" "$cfg"
  done
done
for cfg in "--pack-on draw" "--pack-on count"; do
  timeout -k 10 200 python bench.py --config synthetic8192 --steps 30 --warmup 2 --no-cpu-baseline --no-api $cfg > $OUT/ab.json 2> $OUT/ab.err
  python3 -c "import json,sys; d=json.load(open('$OUT/ab.json')); print('cfg5 %-20s %7.2fM/s' % (sys.argv[1], d['value']/1e6))" "$cfg"
done
