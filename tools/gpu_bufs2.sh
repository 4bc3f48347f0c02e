#!/bin/bash
# A/B of the overlap pipeline depth with the non-persistent lane draw (default), default bench workload
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
for rep in 1 2; do
  for nb in ${NBS:-2 3}; do
    timeout -k 10 200 python bench.py --steps 10 --warmup 3 --bufs $nb --no-cpu-baseline > "$OUT/b_bufs.json" 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { echo "bench bufs=$nb rc=$rc"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels']; print('bufs %s %6.1fM/s ms/step %.3f draw alone %.3f in-region %.3f pairs-in-region %.3f' % (sys.argv[2], d['value']/1e6, d['ms_per_step'], k['draw']['ms'], k['draw']['ms_in_timed_region'], k['pairs_mfma']['ms_in_timed_region']))" "$OUT/b_bufs.json" $nb
  done
done
