#!/bin/bash
# parity of the draw kernels + synthetic8192 (config 5 shape) bench, base library vs in-tree
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "draw or parity" > "$OUT/pytest_cfg5.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_cfg5.log"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for lib in "$@"; do
    [ "$lib" = "tree" ] && lib=""
    CSA_LIB=$lib timeout -k 10 200 python bench.py --config synthetic8192 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/b_cfg5.json" 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { echo "bench $lib rc=$rc"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels']; print('%-16s %6.2fM/s draw %.3f ms (%s) pairs %.3f xt %.3f' % (sys.argv[2] or 'tree', d['value']/1e6, k['draw']['ms'], k['draw']['kernel'], k['pairs_mfma']['ms'], k['xt_count']['ms']))" "$OUT/b_cfg5.json" "$lib"
  done
done
