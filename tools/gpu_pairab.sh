#!/bin/bash
# End-to-end A/B of the pair kernel choice (CSA_PAIR_KERNEL unset / 1 = split / 2 = tile) per config.
# Usage (repo root, via gpurun): bash tools/gpu_pairab.sh "sf_e_110 example_large_200"
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
for cfg in $1; do
for rep in $(seq 1 "${REPS:-3}"); do
  for pk in 1 2; do
    CSA_PAIR_KERNEL=$pk timeout -k 10 300 python bench.py --config "$cfg" --steps ${STEPS:-100} --warmup 3 --no-cpu-baseline --no-api \
        > "$OUT/pairab.json" 2> "$OUT/pairab.err"
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $cfg $pk"; tail -3 "$OUT/pairab.err"; exit $rc; }
    python3 -c "
import json,sys; d=json.load(open('$OUT/pairab.json')); k=d['kernels']
print('%-18s pair_kernel=%s %8.2fM/s  draw %.3f / %.3f  pairs %.3f / %.3f' % (sys.argv[1], sys.argv[2], d['value']/1e6, k['draw']['ms'],
      k['draw']['ms_in_timed_region'], k['pairs_mfma']['ms'], k['pairs_mfma']['ms_in_timed_region']))" "$cfg" "$pk"
  done
done; done
