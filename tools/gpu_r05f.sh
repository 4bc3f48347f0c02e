set -u
OUT=gpurun_out/r05f; mkdir -p $OUT
REPS=3 STEPS=400 bash tools/gpu_ab.sh "k0:CSA_LIB=exp/k0/lib.so tree" > $OUT/ab_sf_e_400.txt 2>&1; rc=$?
cat $OUT/ab_sf_e_400.txt; exit $rc
