"""Host-side timeline of legacy_probabilities (diagnostic, GPU box): wall-clock marks around the
call's stages (encode lookup, pipeline, buffer set-up, kernel enqueue, the one host wait, result
building), best of several calls.  Usage: python tools/api_host_profile.py [instance] [k] [S] [reps]"""
import functools
import importlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
P = importlib.import_module("citizensassemblies-replication_amd")
A = importlib.import_module("citizensassemblies-replication_amd.analysis")
DV = importlib.import_module("citizensassemblies-replication_amd.device")

MARKS = []


def mark(name):
    MARKS.append((name, time.perf_counter()))


def wrap(obj, attr, label):
    f = getattr(obj, attr)

    @functools.wraps(f)
    def g(*a, **k):
        mark(label + ">")
        try:
            return f(*a, **k)
        finally:
            mark(label + "<")
    setattr(obj, attr, g)


if __name__ == "__main__":
    import torch
    name = sys.argv[1] if len(sys.argv) > 1 else "sf_e_110"
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 110
    S = int(sys.argv[3]) if len(sys.argv) > 3 else 10 ** 6
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    d = os.path.join(REPO, "tests", "golden", "instances", name)
    inst = P.read_instance(os.path.join(d, "categories.csv"), os.path.join(d, "respondents.csv"), k)
    wrap(A, "encode_cached", "encode")
    wrap(A, "cached_pipeline", "pipeline")
    wrap(A, "reset_draw_stats", "reset_stats")
    wrap(DV.DevicePipeline, "draw_count_chunks", "enqueue_draw_count")
    wrap(DV.DevicePipeline, "reset", "pipe_reset")
    wrap(A, "finish", "finish")
    wrap(torch.Tensor, "cpu", "host_wait")
    best = None
    for rep in range(reps + 1):
        torch.cuda.synchronize()
        MARKS.clear()
        mark("call>")
        A.legacy_probabilities(inst, S, 0)
        mark("call<")
        t0 = MARKS[0][1]
        rel = [(n, round((t - t0) * 1e3, 4)) for n, t in MARKS]
        if rep and (best is None or rel[-1][1] < best[-1][1]):
            best = rel
    print(json.dumps({"instance": name, "panels": S, "best_call_marks_ms": best}))
