cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pairs.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pairs_r03d.log 2>&1; rc=$?; tail -4 gpurun_out/pairs_r03d.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/pair_bench.py --n 8192 --panels 1000000 > gpurun_out/pairbench_8192_r03d.log 2>&1; rc=$?; tail -3 gpurun_out/pairbench_8192_r03d.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/pair_bench.py --n 1727 --panels 1000000 > gpurun_out/pairbench_1727_r03d.log 2>&1; rc=$?; tail -3 gpurun_out/pairbench_1727_r03d.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config synthetic8192 --steps 20 --no-cpu-baseline --no-api > gpurun_out/bench_r03d_s8192.json 2> gpurun_out/bench_r03d_s8192.err; rc=$?; cut -c1-400 gpurun_out/bench_r03d_s8192.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 200 --no-cpu-baseline --no-api > gpurun_out/bench_r03d_sfe.json 2> gpurun_out/bench_r03d_sfe.err; rc=$?; cut -c1-400 gpurun_out/bench_r03d_sfe.json; exit $rc
