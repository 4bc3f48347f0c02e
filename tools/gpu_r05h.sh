set -u
OUT=gpurun_out/r05h; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "wide or synthetic8192 or parity or draw or layouts or devices" > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=3 STEPS=20 bash tools/gpu_ab.sh "k0:CSA_LIB=exp/k0/lib.so tree" --config synthetic8192 > $OUT/ab_syn.txt 2>&1; rc=$?; cat $OUT/ab_syn.txt; [ $rc -eq 0 ] || exit $rc
