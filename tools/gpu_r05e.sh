set -u
OUT=gpurun_out/r05e; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "api or pair or rows or distributed or rccl or mt_product or parity" > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for spec in "sf_e_110 110 1000000" "example_large_200 200 1250000"; do set -- $spec
  timeout -k 10 300 python tools/api_ab.py $1 $2 $3 8 > $OUT/api_$1.json 2> $OUT/api_$1.err || { tail -5 $OUT/api_$1.err; exit 1; }
  cat $OUT/api_$1.json
done
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit $?
python3 -c "import json; d=json.loads([l for l in open('$OUT/bench.json') if l.startswith('{')][-1]); print(d['value']/1e6, d['ms_per_step'], json.dumps(d.get('api')))"
