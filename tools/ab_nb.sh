#!/bin/bash
# config 5: the pair tile kernel's NB = 4 (512-register waves, default) vs NB = 2 (221 registers: a draw
# wave can share its SIMD) inside the pipelined step, interleaved runs
set -u
O=gpurun_out/r06_ab_nb; mkdir -p $O
for i in 1 2; do
  for nb in 4 2; do
    CSA_P2_NB=$nb timeout -k 10 200 python bench.py --config synthetic8192 --steps 20 --warmup 2 --no-cpu-baseline --no-api > $O/nb$nb.$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.loads([l for l in open('$O/nb$nb.$i.json') if l.startswith('{')][-1]);k=d['kernels'];print('NB=$nb run $i', round(d['value']/1e6,2), round(d['ms_per_step'],2), 'draw', round(k['draw']['ms_in_timed_region'],2), 'pairs', round(k['pairs_mfma']['ms_in_timed_region'],2), 'alone', round(k['pairs_mfma']['ms'],2))"
  done
done
