#!/bin/bash
# A/B of library builds on the default bench (CSA_LIB selects the .so): each library REPS times,
# interleaved, one bench line each (value + draw kernel alone / in the timed region).
# Usage (repo root, via gpurun):  bash tools/gpu_ab_libs.sh "exp/libbase.so citizensassemblies-replication_amd/libcsa_legacy.so" [bench args]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
LIBS=$1; shift || true
REPS=${REPS:-2}
for rep in $(seq 1 "$REPS"); do
  for lib in $LIBS; do
    CSA_LIB=$ROOT/$lib timeout -k 10 200 python bench.py --steps ${STEPS:-200} --warmup 3 --no-cpu-baseline --no-api "$@" \
        > "$OUT/ab.json" 2> "$OUT/ab.err"
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $lib"; tail -3 "$OUT/ab.err"; exit $rc; }
    python3 -c "
import json,sys; d=json.load(open('$OUT/ab.json')); k=d['kernels']; c=d['checks']
print('%-48s %7.2fM/s  draw %.3f / %.3f  pack %.3f  pairs %.3f  checks %s' % (sys.argv[1], d['value']/1e6, k['draw']['ms'],
      k['draw']['ms_in_timed_region'], k.get('pack', {}).get('ms', 0), k.get('pairs_mfma', {}).get('ms', 0),
      (c['last_step_unique'], c['last_step_count_sum'], c['last_step_pair_sum'])))" "$lib"
  done
done
