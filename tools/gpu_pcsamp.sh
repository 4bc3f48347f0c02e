#!/bin/bash
# PC sampling (rocprofv3 host_trap, beta) of a short default bench run: where the draw kernel's waves are
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/pcs_${1:-sfe}; mkdir -p "$OUT"; shift || true
export TMPDIR=/tmp; cd /tmp
timeout -k 10 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
    --pc-sampling-interval ${PCS_INTERVAL:-100} -d "$OUT" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-api --iso-steps 0 "$@" > "$OUT/bench.json" 2> "$OUT/err.log"
rc=$?; echo "rc=$rc"; ls -R "$OUT" | head -20; tail -5 "$OUT/err.log"; exit $rc
