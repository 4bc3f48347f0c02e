#!/bin/bash
# A/B of environment settings on the bench, interleaved REPS times, one summary line each.
# Entries are LABEL:VAR=VALUE[,VAR=VALUE...] (LABEL alone = no extra environment).
# Usage (repo root, via gpurun):  REPS=3 bash tools/gpu_ab_env.sh "tile split:CSA_PAIR_KERNEL=1" [bench args]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
ENTRIES=$1; shift || true
REPS=${REPS:-2}
for rep in $(seq 1 "$REPS"); do
  for ent in $ENTRIES; do
    label=${ent%%:*}; envs=""; [ "$label" != "$ent" ] && envs=${ent#*:}
    ( IFS=','; for kv in $envs; do export "$kv"; done
      timeout -k 10 200 python bench.py --steps ${STEPS:-200} --warmup 3 --no-cpu-baseline --no-api "$@" \
          > "$OUT/ab.json" 2> "$OUT/ab.err" )
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $ent"; tail -3 "$OUT/ab.err"; exit $rc; }
    python3 -c "
import json,sys; d=json.load(open('$OUT/ab.json')); k=d['kernels']; c=d['checks']
print('%-40s %8.2fM/s  draw %.3f/%.3f  pairs %.3f/%.3f  checks %s' % (sys.argv[1], d['value']/1e6, k['draw']['ms'],
      k['draw']['ms_in_timed_region'], k['pairs_mfma']['ms'], k['pairs_mfma']['ms_in_timed_region'],
      (c['last_step_unique'], c['last_step_count_sum'], c['last_step_pair_sum'])))" "$ent"
  done
done
