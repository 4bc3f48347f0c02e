#!/bin/bash
# A/B pair-kernel variants: pair tests, then bench per config for each "ENV=VAL ..." setting.
# Usage: bash tools/gpu_pairab.sh TAG "CSA_PAIR_KB=4" "CSA_PAIR_KB=8" ...
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
TAG=${1:-pab}; shift
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pair" > "$OUT/pytest_$TAG.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_$TAG.log"; [ $rc -eq 0 ] || exit $rc
for setting in "$@"; do
  for c in ${CFGS:-sf_e_110 synthetic8192}; do
    env $setting timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/b_${TAG}.json" 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || exit $rc
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels']['pairs_mfma']; print('%-16s %-22s pairs %.3f ms util %.3f' % (sys.argv[2], sys.argv[3], k['ms'], k['mfma_util']))" "$OUT/b_${TAG}.json" $c "$setting"
  done
done
