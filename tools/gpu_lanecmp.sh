#!/bin/bash
# Draw-kernel layouts: parity tests for all layouts, then one bench per "ENV=VAL" setting.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
TAG=${1:-lc}; shift
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "draw" > "$OUT/pytest_$TAG.log" 2>&1
rc=$?; tail -4 "$OUT/pytest_$TAG.log"; [ $rc -eq 0 ] || exit $rc
for setting in "$@"; do
  env $setting timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/b_${TAG}.json" 2>/dev/null
  rc=$?; [ $rc -eq 0 ] || { echo "bench $setting rc=$rc"; exit $rc; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels']; print('%-20s %6.1fM/s draw %.3f ms (%s) pairs %.3f' % (sys.argv[2], d['value']/1e6, k['draw']['ms'], k['draw']['kernel'], k['pairs_mfma']['ms']))" "$OUT/b_${TAG}.json" "$setting"
done
