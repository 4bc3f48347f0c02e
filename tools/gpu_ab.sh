#!/bin/bash
# A/B runner for the GPU box: optional pytest subset first, then every ENTRY REPS times, interleaved,
# one bench line each, summarised in one row (value, draw / pairs alone and in the timed region, the
# last step's checks).  An ENTRY is LABEL or LABEL:VAR=VALUE[,VAR=VALUE...]; the variables go to that
# bench run only -- CSA_LIB=exp/lib.so (a library build), CSA_DRAW_KERNEL=solo|lane|wide|16|64,
# CSA_PAIR_KERNEL=1|2, CSA_P2_NB=2|4, CSA_DRAW_LDS_PAD=bytes, ...  Extra arguments go to bench.py.
# Every GPU step has its own time limit; a failing step ends the script with its exit code.
# Usage (repo root, via gpurun):
#   REPS=2 STEPS=100 PYTEST="-k pair" bash tools/gpu_ab.sh "base:CSA_LIB=exp/libbase.so tree" --config synthetic8192
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
ENTRIES=$1; shift || true
if [ -n "${PYTEST:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread $PYTEST \
      > "$OUT/pytest_ab.log" 2>&1
  rc=$?; tail -2 "$OUT/pytest_ab.log"; [ $rc -eq 0 ] || exit $rc
fi
for rep in $(seq 1 "${REPS:-2}"); do
  for ent in $ENTRIES; do
    label=${ent%%:*}; envs=""; [ "$label" != "$ent" ] && envs=${ent#*:}
    ( IFS=','; for kv in $envs; do export "$kv"; done
      timeout -k 10 300 python bench.py --steps ${STEPS:-100} --warmup 3 --no-cpu-baseline --no-api "$@" \
          > "$OUT/ab_$label.json" 2> "$OUT/ab_$label.err" )
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $ent"; tail -3 "$OUT/ab_$label.err"; exit $rc; }
    python3 -c "
import json, sys
d = json.loads([ln for ln in open(sys.argv[1]) if ln.startswith('{')][-1]); k = d['kernels']; c = d['checks']
p = k.get('pairs_mfma', {})
print('%-28s %8.2f M/s  draw %.3f / %.3f  pairs %.3f / %.3f  %s  unique %d counts %s' % (sys.argv[2], d['value'] / 1e6,
      k['draw']['ms'], k['draw']['ms_in_timed_region'], p.get('ms', 0), p.get('ms_in_timed_region', 0),
      k['draw']['kernel'], c['last_step_unique'], c['last_step_counts_sha256'][:12]))" "$OUT/ab_$label.json" "$ent"
  done
done
