#!/bin/bash
# GPU box, repo root: the GPU test suite, then the API call A/B (tools/api_ab.py) and the sharded call's
# per-call cost (tools/dist_call_bench.py).  Each step has its own time limit; the first failure ends it.
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_check.log 2>&1; rc=$?
tail -2 gpurun_out/t_check.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/api_ab.py sf_e_110 110 1000000 10 | tail -1 || exit 1
mkdir -p gpurun_out/dist_check
timeout -k 10 300 python tools/dist_call_bench.py > gpurun_out/dist_check/dist_call.json 2> gpurun_out/dist_check/dist_call.err; rc=$?
tail -1 gpurun_out/dist_check/dist_call.json | cut -c1-1500; exit $rc
