#!/bin/bash
# the CSA_PAIR_ALONE block threshold: split vs tile4 alone between 10^4 and 10^6 panels at the two-lane /
# one-lane pool sizes (n = 1727 sf_e, n = 2000 example_large_200)
set -u
O=${1:-gpurun_out/r06_pair_alone}; mkdir -p $O
for n in 1727 2000; do
  for S in 65536 131072 262144 524288; do
    timeout -k 10 120 python tools/pair_bench.py --n $n --panels $S --reps 7 --variants tile4,split --density 0.064 \
      > $O/mid_n${n}_S${S}.log 2>&1 || exit $?
    python -c "import json;d=json.loads(open('$O/mid_n${n}_S${S}.log').read().strip().splitlines()[-1]);v=d['variants'];print($n,$S,round(v['tile4']['ms'],4),round(v['split']['ms'],4))"
  done
done
