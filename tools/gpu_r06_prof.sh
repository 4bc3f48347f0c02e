#!/bin/bash
# Round-6 evidence pass (GPU box, repo root): the default bench line, a rocprofv3 kernel trace of that
# exact command, and the PMC passes per BASELINE shape (tools/gpu_prof.sh) for the committed sources.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/${R06TAG:-r06p}; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 400 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit $?
cut -c1-300 "$OUT/bench_default.json"
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_default" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --no-cpu-baseline > "$OUT/bench_under_rocprof.json" 2> "$OUT/bench_under_rocprof.err" ) || exit $?
echo "[trace] ok"
for cfg in sf_e_110 example_large_200 synthetic8192; do
  bash tools/gpu_prof.sh "${R06TAG:-r06p}_$cfg" --config $cfg > "$OUT/prof_$cfg.log" 2>&1 || { tail -5 "$OUT/prof_$cfg.log"; exit 1; }
  echo "[prof $cfg] ok"
done
echo done
