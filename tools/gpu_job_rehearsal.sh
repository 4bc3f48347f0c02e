#!/bin/bash
# Strong-scaling rehearsal of BASELINE configs 3 and 5 on one GPU: bench.py --job-panels P at N = 1
# and as 2 gloo ranks on the same GPU (RCCL refuses two ranks on one device); the digests of the
# final count vector and pair triangle, the distinct count and the draw statistics must agree.
# Usage (repo root, via gpurun):  bash tools/gpu_job_rehearsal.sh TAG [P_config3] [P_config5]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
TAG=${1:-job}; P3=${2:-10000000}; P5=${3:-4000000}
LOG=$OUT/job_rehearsal_$TAG.log; : > "$LOG"
for spec in "example_large_200 $P3" "synthetic8192 $P5"; do
  set -- $spec; cfg=$1; P=$2
  for n in 1 2; do
    env_extra=""; [ $n -gt 1 ] && env_extra="CSA_BENCH_BACKEND=gloo"
    env $env_extra timeout -k 10 500 python bench.py --config $cfg --job-panels $P --gpus $n --warmup 2 \
        --no-cpu-baseline --no-api > "$OUT/job_${TAG}_${cfg}_n$n.json" 2> "$OUT/job_${TAG}_${cfg}_n$n.err"
    rc=$?; [ $rc -eq 0 ] || { echo "[$cfg n=$n] rc=$rc"; tail -5 "$OUT/job_${TAG}_${cfg}_n$n.err"; exit $rc; }
    python3 -c "
import json, sys
d = json.loads([ln for ln in open(sys.argv[1]) if ln.startswith('{')][-1]); c = d['checks']
print('%-18s n=%d P=%d  %.3f s  %.2f M panels/s  unique %d  counts %s  pairs %s  stats %s' % (sys.argv[2], d['n_gpus'],
      d['config']['job_panels'], d['job_seconds'], d['value'] / 1e6, c['job_unique'], c['job_counts_sha256'][:16],
      (c.get('job_pairs_triu_sha256') or '-')[:16], json.dumps(d['draw_stats'])))" "$OUT/job_${TAG}_${cfg}_n$n.json" $cfg >> "$LOG" \
        || { echo "[$cfg n=$n] no result line"; exit 1; }
    tail -1 "$LOG"
  done
done
