cd $GRAFT_REPO_ROOT; OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "draw or parity or address" > $OUT/pytest_w.log 2>&1; rc=$?; tail -3 $OUT/pytest_w.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config synthetic8192 --steps 20 --warmup 2 --no-cpu-baseline --no-api > $OUT/b_cfg5.json 2> $OUT/b_cfg5.err; rc=$?; echo cfg5 rc=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 3 --no-cpu-baseline --no-api > $OUT/b_sfe.json 2> $OUT/b_sfe.err; echo sfe rc=$?
