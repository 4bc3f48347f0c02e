#!/bin/bash
# Round-6 final evidence (GPU box, repo root): the GPU test suite, smoke(), the default bench line (PMC
# matched to the sources), one 20-step line per BASELINE config and the two --job-panels jobs (configs 3, 5).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; T=${R06TAG:-r06f}; OUT=$ROOT/gpurun_out/$T; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -20 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 400 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit $?
cut -c1-200 "$OUT/bench_default.json"
bash tools/gpu_configs.sh $T > "$OUT/configs.log" 2>&1 || { tail -5 "$OUT/configs.log"; exit 1; }
cat "$OUT/configs.log"
timeout -k 10 200 python bench.py --config example_large_200 --job-panels 10000000 --warmup 3 --no-cpu-baseline --no-api > "$OUT/bench_job3.json" 2> "$OUT/bench_job3.err" || exit $?
timeout -k 10 300 python bench.py --config synthetic8192 --job-panels 100000000 --warmup 3 --no-cpu-baseline --no-api > "$OUT/bench_job5.json" 2> "$OUT/bench_job5.err" || exit $?
python -c "
import json
for f in ['$OUT/bench_job3.json', '$OUT/bench_job5.json']:
    d = json.loads([l for l in open(f) if l.startswith('{')][-1]); print(f, round(d['value'] / 1e6, 2), 'M/s', round(d['job_seconds'], 4), 's')"
echo done
