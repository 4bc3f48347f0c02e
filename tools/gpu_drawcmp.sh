#!/bin/bash
# Compare draw-kernel group sizes: parity tests (default config) + bench per CSA_DRAW_GROUP.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
TAG=${1:-dc}; shift || true; GL=${1:-16 8 4}; shift || true
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "parity or pairs or draw" > "$OUT/pytest_$TAG.log" 2>&1
rc=$?; tail -8 "$OUT/pytest_$TAG.log"; echo "[pytest] rc=$rc"
[ $rc -eq 0 ] || exit $rc
for g in $GL; do
  CSA_DRAW_GROUP=$g timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > "$OUT/bench_${TAG}_g$g.json" 2> "$OUT/bench_${TAG}_g$g.err"
  rc=$?; echo "[bench G=$g] rc=$rc"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels']; print('G=%s value %.1fM/s draw %.2f ms pairs %.3f ms' % (sys.argv[2], d['value']/1e6, k['draw']['ms'], k.get('pairs_mfma',{}).get('ms',0)))" "$OUT/bench_${TAG}_g$g.json" $g || tail -5 "$OUT/bench_${TAG}_g$g.err"
  [ $rc -eq 0 ] || exit $rc
done
