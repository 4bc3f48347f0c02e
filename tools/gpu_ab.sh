#!/bin/bash
# A/B of library builds x draw-kernel layouts on the default bench, interleaved REPS times, one
# summary line each.  Entries are LIB or LIB:LAYOUT (LAYOUT -> CSA_DRAW_KERNEL, e.g. solo|lane).
# Usage (repo root, via gpurun):
#   bash tools/gpu_ab.sh "exp/libbase.so citizensassemblies-replication_amd/libcsa_legacy.so:solo" [bench args]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
ENTRIES=$1; shift || true
REPS=${REPS:-2}
for rep in $(seq 1 "$REPS"); do
  for ent in $ENTRIES; do
    lib=${ent%%:*}; lay=""; [ "$lib" != "$ent" ] && lay=${ent#*:}
    CSA_LIB=$ROOT/$lib CSA_DRAW_KERNEL=$lay timeout -k 10 200 python bench.py --steps ${STEPS:-200} --warmup 3 \
        --no-cpu-baseline --no-api "$@" > "$OUT/ab.json" 2> "$OUT/ab.err"
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $ent"; tail -3 "$OUT/ab.err"; exit $rc; }
    python3 -c "
import json,sys; d=json.load(open('$OUT/ab.json')); k=d['kernels']; c=d['checks']
print('%-56s %7.2fM/s  draw %.3f / %.3f  checks %s' % (sys.argv[1], d['value']/1e6, k['draw']['ms'],
      k['draw']['ms_in_timed_region'], (c['last_step_unique'], c['last_step_count_sum'], c['last_step_pair_sum'])))" "$ent"
  done
done
