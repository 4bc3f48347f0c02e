set -u
OUT=gpurun_out/r05g; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/dist_call_bench.py 1250000 12500000 5 > $OUT/dist_call.json 2> $OUT/dist_call.err || { tail -5 $OUT/dist_call.err; exit 1; }
for spec in "example_large_200 1250000" "synthetic8192 12500000"; do set -- $spec
  timeout -k 10 300 python bench.py --config $1 --job-panels $2 --warmup 2 --no-cpu-baseline --no-api > $OUT/job_$1.json 2> $OUT/job_$1.err || exit $?
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['job_seconds']*1e3, 'ms', d['value']/1e6)" $OUT/job_$1.json
done
python3 -c "
import json; d=json.load(open('$OUT/dist_call.json'))
for c in ('config3_share','config5_share'):
  for m,v in d[c].items():
    if isinstance(v, dict): print(c, m, v['calls_ms'], v['best'])"
REPS=2 STEPS=400 bash tools/gpu_ab.sh "k0:CSA_LIB=exp/k0/lib.so tree" > $OUT/ab.txt 2>&1; rc=$?; cat $OUT/ab.txt; [ $rc -eq 0 ] || exit $rc
bash tools/clock_sample.sh
