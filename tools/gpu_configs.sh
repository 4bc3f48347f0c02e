#!/bin/bash
# Bench every BASELINE config on one GPU (no CPU baseline); one JSON line per config.
# Usage: bash tools/gpu_configs.sh TAG [configs...]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
TAG=${1:-cf}; shift || true
CFGS=${*:-sf_e_110 example_large_200 synthetic8192 example_small_20 couples}
for c in $CFGS; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 2 --no-cpu-baseline --no-api > "$OUT/bench_${TAG}_$c.json" 2> "$OUT/bench_${TAG}_$c.err"
  rc=$?; echo "[bench $c] rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$OUT/bench_${TAG}_$c.err"; exit $rc; }
  python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels']
print('%-18s %8.2fM/s step %.2f ms | ' % (sys.argv[2], d['value']/1e6, d['ms_per_step']) + ' '.join('%s %.3f' % (s, v['ms']) for s, v in k.items()) + ' | %s' % k['draw']['kernel'])" "$OUT/bench_${TAG}_$c.json" $c
done
