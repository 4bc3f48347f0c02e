#!/bin/bash
# int8 engine re-measured on these sources (split kernel; the tile kernel is fp4-only), fp4 beside it
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
for n in 8192 1727; do
  for eng in i8 fp4; do
    v=split; [ $eng = fp4 ] && v=split,tile2
    timeout -k 10 150 python tools/pair_bench.py --n $n --engine $eng --variants $v --reps 5 > "$OUT/pb_${eng}_$n.json" 2> "$OUT/pb_${eng}_$n.err" || { echo "pair_bench $eng $n failed"; tail -3 "$OUT/pb_${eng}_$n.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], {k: (round(v['ms'],3), round(v['frac'],3)) for k, v in d['variants'].items()})" "$OUT/pb_${eng}_$n.json" $eng $n
  done
done
