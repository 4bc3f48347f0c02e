#!/bin/bash
# A/B: draw grid (CSA_DRAW_WAVES) x counting-stream priority (CSA_BENCH_PRIO), default bench workload
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_w2.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_w2.log"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for cfg in "0 1" "0 0" "1 1" "1 0"; do
    set -- $cfg
    CSA_DRAW_WAVES=$1 CSA_BENCH_PRIO=$2 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/b_w2.json" 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { echo "bench $cfg rc=$rc"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels']; print('waves/prio %s %6.1fM/s ms/step %.3f draw alone %.3f in-region %.3f pairs-in-region %.3f' % (sys.argv[2], d['value']/1e6, d['ms_per_step'], k['draw']['ms'], k['draw']['ms_in_timed_region'], k['pairs_mfma']['ms_in_timed_region']))" "$OUT/b_w2.json" "$cfg"
  done
done
