cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r03j}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_$T.log; [ $rc -eq 0 ] || exit $rc
for c in synthetic8192 sf_e_110 example_large_200; do
  st=200; [ $c = synthetic8192 ] && st=20
  timeout -k 10 300 python -u bench.py --config $c --steps $st --no-cpu-baseline --no-api > gpurun_out/bench_${T}_$c.json 2> gpurun_out/bench_${T}_$c.err; rc=$?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/bench_${T}_$c.json')); k=d['kernels']; print('$c', round(d['value']/1e6,2), 'M/s', {n: round(v.get('ms_in_timed_region',0),3) for n,v in k.items()}, 'alone', {n: round(v.get('ms',0),3) for n,v in k.items()})"
  [ $rc -eq 0 ] || exit $rc
done
