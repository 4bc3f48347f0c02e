cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r03l}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_$T.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab.sh "exp/libbase.so citizensassemblies-replication_amd/libcsa_legacy.so" || exit 1
REPS=1 bash tools/gpu_ab.sh "exp/libbase.so citizensassemblies-replication_amd/libcsa_legacy.so" --config example_large_200 || exit 1
REPS=1 bash tools/gpu_ab.sh "exp/libbase.so citizensassemblies-replication_amd/libcsa_legacy.so" --config example_small_20 || exit 1
