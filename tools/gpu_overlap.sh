#!/bin/bash
# bench with and without the overlapped draw stream, alternating
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
TAG=${1:-ov}; shift || true
for rep in 1 2; do
  for mode in "--no-overlap" ""; do
    timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $mode "$@" > "$OUT/b_${TAG}.json" 2> "$OUT/b_${TAG}.err"
    rc=$?; [ $rc -eq 0 ] || { echo "bench $mode rc=$rc"; tail -5 "$OUT/b_${TAG}.err"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels']; print('%-14s %6.1fM/s %.3f ms/step draw %.3f hash %.3f xt %.3f pairs %.3f uniq %.3f checks %s' % (sys.argv[2] or 'overlap', d['value']/1e6, d['ms_per_step'], k['draw']['ms'], k['hash']['ms'], k['xt_count']['ms'], k['pairs_mfma']['ms'], k['unique']['ms'], d['checks']))" "$OUT/b_${TAG}.json" "$mode"
  done
done
