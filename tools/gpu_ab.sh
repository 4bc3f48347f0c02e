#!/bin/bash
# A/B of two library builds on the bench (CSA_LIB=exp/libbase.so vs the in-tree build), alternating.
# Usage: bash tools/gpu_ab.sh TAG [pytest -k expr]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
TAG=${1:-ab}; KEXPR=${2:-draw}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$KEXPR" > "$OUT/pytest_$TAG.log" 2>&1
rc=$?; tail -4 "$OUT/pytest_$TAG.log"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for lib in exp/libbase.so ""; do
    CSA_LIB=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/b_${TAG}.json" 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { echo "bench $lib rc=$rc"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels']; print('%-16s %6.1fM/s draw %.3f ms (%s) pairs %.3f' % (sys.argv[2] or 'new', d['value']/1e6, k['draw']['ms'], k['draw']['kernel'], k['pairs_mfma']['ms']))" "$OUT/b_${TAG}.json" "$lib"
  done
done
