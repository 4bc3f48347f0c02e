#!/bin/bash
# Rehearse bench.py's N > 1 path on a 1-GPU box: 2 ranks on cuda:0 over gloo (RCCL refuses two
# ranks on one device), and compare the whole-job checks with a 1-rank run of the same panels.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
P=${1:-200000}
CFG=${2:-sf_e_110}
timeout -k 10 300 python bench.py --config $CFG --steps 20 --warmup 2 --no-cpu-baseline --no-api --panels $((2 * P)) > "$OUT/reh_n1.json" 2> "$OUT/reh_n1.err"
rc=$?; echo "[n1] rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/reh_n1.err"; exit $rc; }
CSA_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --config $CFG --gpus 2 --steps 20 --warmup 2 --no-cpu-baseline \
    --no-api --panels $P > "$OUT/reh_n2.json" 2> "$OUT/reh_n2.err"
rc=$?; echo "[n2] rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/reh_n2.err"; exit $rc; }
python3 - "$OUT/reh_n1.json" "$OUT/reh_n2.json" <<'PY'
import json, sys
a = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print("n1", a["checks"], "value %.1fM" % (a["value"] / 1e6))
print("n2", b["checks"], "value %.1fM" % (b["value"] / 1e6), "exchange ms", b["kernels"].get("exchange"),
      "draw stream busy %.3f" % b["draw_stream_busy"])
assert a["checks"] == b["checks"], "N=2 rehearsal differs from N=1"
print("checks match")
PY
