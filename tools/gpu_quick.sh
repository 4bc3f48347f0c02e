#!/bin/bash
# Quick GPU loop: a pytest subset (-k expression), then every config's bench line.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
TAG=${1:-q}; KEXPR=${2:-}
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$KEXPR" > "$OUT/pytest_$TAG.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest_$TAG.log"; echo "[pytest] rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
bash tools/gpu_configs.sh "$TAG" ${CFGS:-}
