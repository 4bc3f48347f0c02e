set -u
OUT=gpurun_out/r05c; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for n in 1727 2000; do for lib in exp/libpbase.so exp/libppipe.so; do
  CSA_LIB=$lib timeout -k 10 120 python tools/pair_bench.py --n $n --variants split --reps 5 > $OUT/pair_${n}_$(basename $lib).jsonl 2>&1 || exit 1
  echo "$n $lib $(grep '^split' $OUT/pair_${n}_$(basename $lib).jsonl)"
done; done
REPS=3 STEPS=100 bash tools/gpu_ab.sh "k0:CSA_LIB=exp/k0/lib.so k1:CSA_LIB=exp/k1/lib.so" > $OUT/ab_k8.txt 2>&1; rc=$?
cat $OUT/ab_k8.txt; exit $rc
