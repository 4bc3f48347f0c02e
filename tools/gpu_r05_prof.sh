#!/bin/bash
# Round-5 evidence pass (GPU box, repo root): the default bench line, a rocprofv3 kernel trace of that
# exact command, PMC passes per BASELINE shape, the VALU-region counts of the stamps build, and the
# config-5 clock probe (draw alone / pairs alone / the pipelined step, clock = GRBM_GUI_ACTIVE / 8 / duration).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/${R05TAG:-r05p}; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 400 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit $?
cut -c1-400 "$OUT/bench_default.json"
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_default" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --no-cpu-baseline > "$OUT/bench_under_rocprof.json" 2> "$OUT/bench_under_rocprof.err" ) || exit $?
echo "[trace] ok"
for cfg in sf_e_110 example_large_200 synthetic8192; do
  bash tools/gpu_prof.sh "r05_$cfg" --config $cfg > "$OUT/prof_$cfg.log" 2>&1 || { tail -5 "$OUT/prof_$cfg.log"; exit 1; }
  echo "[prof $cfg] ok"
done
CSA_LIB=exp/libstamps.so timeout -k 10 200 python tools/lane_stamps.py --config sf_e_110 > "$OUT/lane_stamps_sf_e_110.json" 2> "$OUT/lane_stamps.err" || exit $?
echo "[stamps] ok"
cd /tmp
P=$OUT/clock
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU -d "$P/draw_only" -o run --output-format csv -- python3 "$ROOT/bench.py" --config synthetic8192 --no-pairs --steps 5 --warmup 1 --iso-steps 0 --no-cpu-baseline --no-api > "$P.draw_only.json" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -d "$P/pairs_only" -o run --output-format csv -- python3 "$ROOT/tools/pair_bench.py" --n 8192 --variants tile4 --reps 4 > "$P.pairs_only.json" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU -d "$P/step" -o run --output-format csv -- python3 "$ROOT/bench.py" --config synthetic8192 --steps 5 --warmup 1 --iso-steps 0 --no-cpu-baseline --no-api > "$P.step.json" 2>&1 || exit $?
echo done
