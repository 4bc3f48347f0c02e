cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r03g}
timeout -k 10 400 python -u -m pytest tests/test_gpu_pairs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pairs_$T.log 2>&1; rc=$?; tail -3 gpurun_out/pairs_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/pair_bench.py --n 8192 --panels 1000000 > gpurun_out/pairbench_8192_$T.log 2>&1; rc=$?; head -2 gpurun_out/pairbench_8192_$T.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/pair_bench.py --n 1727 --panels 1000000 > gpurun_out/pairbench_1727_$T.log 2>&1; rc=$?; head -2 gpurun_out/pairbench_1727_$T.log | cut -c1-200; exit $rc
