#!/bin/bash
# VALU mixed-stream table; draw parity; A/B (HEAD library vs tree) at sf_e and synthetic8192
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 120 tools/valu_rate enc > "$OUT/valu_enc_r03.jsonl" || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_draw.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_r03n.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_r03n.log"; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_libs.sh "exp/libprev.so citizensassemblies-replication_amd/libcsa_legacy.so" || exit $?
for rep in 1 2; do
  for lib in exp/libprev.so citizensassemblies-replication_amd/libcsa_legacy.so; do
    CSA_LIB=$ROOT/$lib timeout -k 10 200 python bench.py --config synthetic8192 --steps 3 --warmup 1 --no-cpu-baseline --no-api > "$OUT/b_cfg5.json" 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { echo "bench $lib rc=$rc"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels']; print('%-50s %6.2fM/s draw %.3f ms pairs %.3f' % (sys.argv[2], d['value']/1e6, k['draw']['ms'], k['pairs_mfma']['ms']))" "$OUT/b_cfg5.json" "$lib"
  done
done
