#!/bin/bash
# kernel-alone times of the split pair kernel (pair_mfma_kernel) vs the per-CU tile kernel
# (pair_fp4_tile_kernel<4>, what CSA_PAIR_ALONE picks) at the pool sizes of the BASELINE configs and at
# legacy_probabilities' chunk sizes (10^4 = the reference's S, 10^6 = one chunk).  Prints one JSON line per case.
set -u
O=${1:-gpurun_out/r06_pair_alone}; mkdir -p $O
for n in 20 200 1727 2000 8192; do
  for S in 10000 1000000; do
    case $n in 20) d=0.1;; 200) d=0.1;; 1727) d=0.064;; 2000) d=0.1;; 8192) d=0.025;; esac
    timeout -k 10 120 python tools/pair_bench.py --n $n --panels $S --reps 5 --variants tile4,split --density $d \
      > $O/n${n}_S${S}.log 2>&1 || exit $?
    tail -1 $O/n${n}_S${S}.log
  done
done
