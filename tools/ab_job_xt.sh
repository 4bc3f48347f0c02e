set -u
O=gpurun_out/r06_ab_job; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_headline.py tests/test_gpu_api.py tests/test_gpu_parity.py -k "xt_ring or job or chunks or distributed or growing or headline or sample_device" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
 for m in draw count; do
  timeout -k 10 120 python bench.py --config example_large_200 --job-panels 10000000 --warmup 3 --no-cpu-baseline --no-api --xt-from $m > $O/job3_$m.$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads([l for l in open('$O/job3_$m.$i.json') if l.startswith('{')][-1]);print('job3 $m $i',round(d['value']/1e6,2),round(d['job_seconds']*1e3,2),'ms')"
  timeout -k 10 120 python bench.py --config sf_e_110 --job-panels 10000000 --warmup 3 --no-cpu-baseline --no-api --xt-from $m > $O/jobsf_$m.$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads([l for l in open('$O/jobsf_$m.$i.json') if l.startswith('{')][-1]);print('jobsf $m $i',round(d['value']/1e6,2),round(d['job_seconds']*1e3,2),'ms')"
 done
done
