set -u
O=gpurun_out/r06_ab_xt; mkdir -p $O
for i in 1 2; do
 for m in draw count; do
  timeout -k 10 200 python bench.py --steps 200 --xt-from $m --no-cpu-baseline --no-api > $O/$m.$i.json 2> $O/$m.$i.err || exit $?
  python -c "import json,sys;d=json.loads([l for l in open('$O/$m.$i.json') if l.startswith('{')][-1]);print('$m',$i,round(d['value']/1e6,2),d['ms_per_step'],d['checks']['last_step_counts_sha256'][:12],d['checks'].get('last_step_pairs_triu_sha256','')[:12],{k:round(v.get('ms_in_timed_region',0),3) for k,v in d['kernels'].items()})"
 done
done
