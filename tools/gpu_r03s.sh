#!/bin/bash
# Round-3 artifacts: parity tests, default bench line (CPU baseline included), kernel trace + PMC passes
# of the default bench, every BASELINE config's bench line
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
bash tools/gpu_round.sh ${1:-r03s} || exit $?
bash tools/gpu_configs.sh ${1:-r03s} example_large_200 synthetic8192 example_small_20 couples || exit $?
