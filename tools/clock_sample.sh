#!/bin/bash
# Config-5 clock probe without a profiler (PMC collection serialises kernels, so it cannot see the
# co-running step): sample the GPU's current SCLK with amd-smi every ~0.25 s while one workload runs
# (the pipelined synthetic8192 step, its draws alone, the pair tile kernel alone), and report the median
# of the busy samples.  Usage (GPU box, repo root): bash tools/clock_sample.sh
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/r05clk; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 5 20 amd-smi metric -g 0 -c > "$OUT/amdsmi_probe.txt" 2>&1; echo "[probe rc=$?]"; head -20 "$OUT/amdsmi_probe.txt"
run() {  # label, command...
  local label=$1; shift
  "$@" > "$OUT/$label.out" 2>&1 &
  local pid=$!
  : > "$OUT/$label.clk"
  while kill -0 $pid 2>/dev/null; do
    timeout -k 2 5 amd-smi metric -g 0 -c --json >> "$OUT/$label.clk" 2>/dev/null
    echo "@@" >> "$OUT/$label.clk"
    sleep 0.2
  done
  wait $pid; echo "[$label rc=$?]"
}
run step timeout -k 10 300 python bench.py --config synthetic8192 --steps 40 --warmup 2 --iso-steps 0 --no-cpu-baseline --no-api
run draw_only timeout -k 10 300 python bench.py --config synthetic8192 --no-pairs --steps 60 --warmup 2 --iso-steps 0 --no-cpu-baseline --no-api
run pairs_only timeout -k 10 300 python tools/pair_bench.py --n 8192 --variants tile4 --reps 80
run sf_e timeout -k 10 300 python bench.py --steps 1500 --warmup 2 --iso-steps 0 --no-cpu-baseline --no-api
echo done
