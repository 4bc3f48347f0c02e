#!/bin/bash
# Bench A/B/n of several library builds (CSA_LIB=<path>; "" = the in-tree build), alternating.
# Usage: bash tools/gpu_abn.sh TAG lib1 lib2 ...
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
TAG=$1; shift
for rep in 1 2; do
  for lib in "$@"; do
    [ "$lib" = "tree" ] && lib=""
    CSA_LIB=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/b_${TAG}.json" 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { echo "bench $lib rc=$rc"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels']; print('%-16s %6.1fM/s draw %.3f ms pairs %.3f' % (sys.argv[2] or 'tree', d['value']/1e6, k['draw']['ms'], k['pairs_mfma']['ms']))" "$OUT/b_${TAG}.json" "$lib"
  done
done
