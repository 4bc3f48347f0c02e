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
rc=$?; echo "[n2 torchrun] rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/reh_n2.err"; exit $rc; }
# bench.py --gpus 2 without a launcher: it starts its two rank processes itself
CSA_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --config $CFG --gpus 2 --steps 20 --warmup 2 --no-cpu-baseline \
    --no-api --panels $P > "$OUT/reh_n2s.json" 2> "$OUT/reh_n2s.err"
rc=$?; echo "[n2 self-launch] rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/reh_n2s.err"; exit $rc; }
python3 - "$OUT/reh_n1.json" "$OUT/reh_n2.json" "$OUT/reh_n2s.json" <<'PY'
import json, sys
KEYS = ("last_step_unique", "last_step_count_sum", "last_step_pair_sum", "last_step_counts_sha256",
        "last_step_pairs_triu_sha256")
a = json.loads([ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1])
print("n1", a["n_gpus"], {k: a["checks"][k] for k in KEYS}, "value %.1fM" % (a["value"] / 1e6))
for f in sys.argv[2:]:
    b = json.loads([ln for ln in open(f) if ln.startswith("{")][-1])
    print("n2", b["n_gpus"], {k: b["checks"][k] for k in KEYS}, "value %.1fM" % (b["value"] / 1e6), "exchange",
          b["kernels"].get("exchange"), "draw stream busy %.3f" % b["draw_stream_busy"], "draw_stats", b["draw_stats"],
          "sample_devices", b["checks"].get("sample_devices"))
    assert b["n_gpus"] == 2
    assert all(a["checks"][k] == b["checks"][k] for k in KEYS), "N=2 rehearsal differs from N=1"
    assert b["checks"]["sample_devices"]["equal_to_rank_sharded"], "csa_legacy_sample_devices differs"
print("checks match")
PY
