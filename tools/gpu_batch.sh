#!/bin/bash
# GPU batch: full -m gpu suite, the N=2 gloo rehearsal of the multi-GPU bench path, every config's bench line.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
TAG=${1:-bt}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > "$OUT/pytest_$TAG.log" 2>&1
rc=$?; tail -4 "$OUT/pytest_$TAG.log"; echo "[pytest] rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_rehearse_multi.sh 200000 > "$OUT/rehearse_$TAG.log" 2>&1; rc=$?; tail -6 "$OUT/rehearse_$TAG.log"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_configs.sh "$TAG"
