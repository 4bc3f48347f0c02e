#!/bin/bash
# XCD window sync of pair_fp4_tile_kernel: pair parity, kernel alone per window, FETCH per window,
# synthetic8192 end to end
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
CSA_P2_SYNC=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_pairs.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_r03p.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_r03p.log"; [ $rc -eq 0 ] || exit $rc
for w in 0 16 32 64 128; do
  CSA_P2_SYNC=$w timeout -k 10 120 python tools/pair_bench.py --variants tile2 --reps 5 > "$OUT/pb_sync$w.json" 2> "$OUT/pb_sync$w.err" || { echo "pair_bench $w failed"; tail -3 "$OUT/pb_sync$w.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('sync', sys.argv[2], {k: (round(v['ms'],3), round(v['frac'],3)) for k, v in d['variants'].items()})" "$OUT/pb_sync$w.json" $w
done
for w in 0 32 64; do
  CSA_P2_SYNC=$w PASSES="pmc_fetch:--pmc FETCH_SIZE|pmc_tcc:--pmc TCC_HIT_sum TCC_MISS_sum" bash tools/gpu_pmc_pair.sh sync$w --variants tile2 || exit $?
done
REPS=2 bash tools/gpu_ab_env.sh "nosync sync32:CSA_P2_SYNC=32 sync64:CSA_P2_SYNC=64" --config synthetic8192 --steps 3 --warmup 1 || exit $?
