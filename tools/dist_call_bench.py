"""Per-call cost of the sharded product path on one GPU: a one-rank RCCL process
group (backend "nccl") with the 24-byte key exchange forced on (CSA_FORCE_EXCHANGE=1, the world > 1
path: packed pair all_reduce, key all_to_alls, owner re-draws, one all_reduce of counts + statistics +
distinct count), then distributed.legacy_probabilities_distributed called repeatedly at one GPU's
share of BASELINE config 3 (1.25e6 example_large_200 panels) and config 5 (1.25e7 synthetic n = 8192
panels).  Every call after the first reuses the cached encoding, pipeline and exchange; the
per-stage host timings (setup / device incl. the one host wait / finish) are printed with the
results' invariants checked.  found_panels keep nothing (they are re-drawn where read), so
keep_panels=True and False cost the same per call; the re-draw itself (found.rows() on this rank,
alone) is timed separately.  Compare with `bench.py --job-panels P` for the same share (the same
kernels without the API).  Prints one JSON line.

Usage (GPU box): python tools/dist_call_bench.py [S_config3] [S_config5] [calls]"""
import json
import os
import socket
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import importlib  # noqa: E402

P = importlib.import_module("citizensassemblies-replication_amd")
A = importlib.import_module("citizensassemblies-replication_amd.analysis")
D = importlib.import_module("citizensassemblies-replication_amd.distributed")


def run(name, k, S, calls, modes):
    import torch
    d = os.path.join(REPO, "tests", "golden", "instances", name)
    inst = P.read_instance(os.path.join(d, "categories.csv"), os.path.join(d, "respondents.csv"), k)
    out = {"instance": name, "k": k, "panels": S}
    for label, kw in modes:
        rows = []
        for c in range(calls):
            torch.cuda.synchronize()
            tm = {}
            t = time.perf_counter()
            alloc, found, hist = D.legacy_probabilities_distributed(inst, S, 0, timings=tm, **kw)
            dt = time.perf_counter() - t
            total = sum(alloc.values())
            assert abs(total - k) < 1e-6 * k, total                      # sum of probabilities = k
            rows.append(dict(tm, call_ms=dt * 1e3))
        redraw_ms = None
        # (the host dedupe of rows() -- np.unique over S rows of W words, as the one-GPU call's -- is the cost
        # past a few GB: timed at the config-3 share only)
        if kw.get("keep_panels", True) and S * ((len(inst.agents) + 63) // 64) <= (64 << 20):
            t = time.perf_counter()
            u = found.rows()
            redraw_ms = (time.perf_counter() - t) * 1e3
            assert len(u) == len(found)
        best = min(rows[1:] or rows, key=lambda r: r["call_ms"])
        out[label] = {"calls_ms": [round(r["call_ms"], 3) for r in rows], "second_call_ms": round(rows[1]["call_ms"], 3)
                      if len(rows) > 1 else None, "best": {k_: round(v, 3) for k_, v in best.items()},
                      "panels_per_s_best": S / (best["call_ms"] / 1e3), "unique": len(found),
                      "stats": A.LAST_RUN_STATS, "found_rows_redraw_ms": redraw_ms}
        print(json.dumps({name: {label: out[label]}}), file=sys.stderr, flush=True)
    return out


if __name__ == "__main__":
    import torch
    import torch.distributed as dist
    s3 = int(sys.argv[1]) if len(sys.argv) > 1 else 1250000
    s5 = int(sys.argv[2]) if len(sys.argv) > 2 else 12500000
    calls = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    os.environ.setdefault("CSA_FORCE_EXCHANGE", "1")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1)
    try:
        res = {"note": "legacy_probabilities_distributed under a 1-rank RCCL group on one MI355X, the n-th call "
                       "(cached encoding / pipeline / exchange); call_ms = host wall time of the call; "
                       "found_rows_redraw_ms = found.rows() after the last call (re-draw of [0, S) + dedupe)",
               "force_exchange": os.environ.get("CSA_FORCE_EXCHANGE"),
               "config3_share": run("example_large_200", 200, s3, calls,
                                    [("no_panels", {"keep_panels": False}), ("keep_panels", {})]),
               "config5_share": run("synthetic8192_200", 200, s5, calls,
                                    [("no_panels", {"keep_panels": False}), ("keep_panels", {})])}
        print(json.dumps(res), flush=True)
    finally:
        dist.destroy_process_group()
