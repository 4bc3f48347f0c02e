set -u
OUT=gpurun_out/r05a; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/dist_call_bench.py > $OUT/dist_call.json 2> $OUT/dist_call.err; rc=$?
tail -c 3000 $OUT/dist_call.err; [ $rc -eq 0 ] || exit $rc
for spec in "example_large_200 1250000" "synthetic8192 12500000"; do set -- $spec
  timeout -k 10 300 python bench.py --config $1 --job-panels $2 --warmup 2 --no-cpu-baseline --no-api > $OUT/job_$1.json 2> $OUT/job_$1.err || exit $?
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['job_seconds'], d['value']/1e6)" $OUT/job_$1.json
done
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit $?
python3 -c "import json; d=json.loads([l for l in open('$OUT/bench.json') if l.startswith('{')][-1]); print(d['value']/1e6, d['ms_per_step'], json.dumps(d.get('api')))"
