#!/bin/bash
# register-transpose xt_count_kernel: full GPU parity, then A/B vs the HEAD library (xt_count alone / in region)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_r03q.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_r03q.log"; [ $rc -eq 0 ] || exit $rc
for cfg in sf_e_110 synthetic8192; do
  for rep in 1 2; do
    for lib in exp/libprev.so citizensassemblies-replication_amd/libcsa_legacy.so; do
      st=200; [ $cfg = synthetic8192 ] && st=3
      CSA_LIB=$ROOT/$lib timeout -k 10 200 python bench.py --config $cfg --steps $st --warmup 2 --no-cpu-baseline --no-api > "$OUT/ab.json" 2> "$OUT/ab.err"
      rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $lib"; tail -3 "$OUT/ab.err"; exit $rc; }
      python3 -c "
import json,sys; d=json.load(open('$OUT/ab.json')); k=d['kernels']; x=k['xt_count']
print('%-14s %-48s %8.2fM/s  xt %.4f / %.4f ms  draw %.3f  checks %s' % ('$cfg', sys.argv[1], d['value']/1e6, x['ms'], x.get('ms_in_timed_region', 0), k['draw']['ms'], (d['checks']['last_step_unique'], d['checks']['last_step_count_sum'], d['checks']['last_step_pair_sum'])))" "$lib"
    done
  done
done
