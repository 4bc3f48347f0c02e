set -u
OUT=gpurun_out/r05d; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/pair_bench.py --n 1727 --variants split,tile4,tile2 --reps 5 > $OUT/pair_1727.jsonl 2>&1 || exit 1
grep -v '^{"n"' $OUT/pair_1727.jsonl | cut -c1-200
for cfg in example_large_200; do
  REPS=2 STEPS=20 bash tools/gpu_ab.sh "k0:CSA_LIB=exp/k0/lib.so tree" --config $cfg > $OUT/ab_$cfg.txt 2>&1; rc=$?
  cat $OUT/ab_$cfg.txt; [ $rc -eq 0 ] || exit $rc
done
REPS=2 STEPS=100 bash tools/gpu_ab.sh "k0:CSA_LIB=exp/k0/lib.so tree" > $OUT/ab_sf_e.txt 2>&1; rc=$?
cat $OUT/ab_sf_e.txt; exit $rc
