set -u
OUT=gpurun_out/r05b; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "api or distributed or rccl or rows or devices or mt_product" > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for spec in "sf_e_110 110 1000000" "example_large_200 200 1250000" "synthetic8192_200 200 1000000"; do set -- $spec
  timeout -k 10 300 python tools/api_ab.py $1 $2 $3 8 > $OUT/api_$1.json 2> $OUT/api_$1.err || { tail -5 $OUT/api_$1.err; exit 1; }
  cat $OUT/api_$1.json
done
timeout -k 10 300 python -u tools/dist_call_bench.py 1250000 12500000 4 > $OUT/dist_call.json 2> $OUT/dist_call.err; rc=$?
python3 -c "
import json; d=json.load(open('$OUT/dist_call.json'))
for c in ('config3_share','config5_share'):
  for m,v in d[c].items():
    if isinstance(v, dict): print(c, m, v['calls_ms'])"
