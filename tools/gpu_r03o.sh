#!/bin/bash
# fp4 MFMA rate table; draw parity; A/B (HEAD library vs tree) at sf_e
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 60 tools/mfma_rate > "$OUT/mfma_rate_r03.jsonl" || exit $?
cat "$OUT/mfma_rate_r03.jsonl"
timeout -k 10 400 python -u -m pytest tests/test_gpu_draw.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_r03o.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_r03o.log"; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_libs.sh "exp/libprev.so citizensassemblies-replication_amd/libcsa_legacy.so" || exit $?
