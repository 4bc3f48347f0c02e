"""A/B of the legacy_probabilities call (analysis.py:162 signature) on one GPU: the chunk plan of
DevicePipeline.draw_count_chunks (the default flat cuts of up to 2^20 panels vs CSA_CHUNK_PLAN=round,
the round-aligned plan), interleaved calls, best and median wall time per call, plus the pair-histogram
materialisation (hist.upper()).  Prints one JSON line.

Usage (GPU box): python tools/api_ab.py [instance] [k] [S] [reps]"""
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import importlib  # noqa: E402

P = importlib.import_module("citizensassemblies-replication_amd")
A = importlib.import_module("citizensassemblies-replication_amd.analysis")

if __name__ == "__main__":
    import torch
    name = sys.argv[1] if len(sys.argv) > 1 else "sf_e_110"
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 110
    S = int(sys.argv[3]) if len(sys.argv) > 3 else 10 ** 6
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    d = os.path.join(REPO, "tests", "golden", "instances", name)
    inst = P.read_instance(os.path.join(d, "categories.csv"), os.path.join(d, "respondents.csv"), k)
    plans = {"round": "round", "flat": None}
    times = {p: [] for p in plans}
    mats = []
    ref = None
    for rep in range(reps + 1):
        for p, env in plans.items():
            if env:
                os.environ["CSA_CHUNK_PLAN"] = env
            else:
                os.environ.pop("CSA_CHUNK_PLAN", None)
            torch.cuda.synchronize()
            t = time.perf_counter()
            alloc, found, hist = A.legacy_probabilities(inst, S, 0)
            dt = time.perf_counter() - t
            t = time.perf_counter()
            up = hist.upper()
            mats.append(time.perf_counter() - t)
            key = (len(found), sum(alloc.values()), float(up.sum()), A.LAST_RUN_STATS["attempts"])
            assert ref is None or key == ref, (key, ref)
            ref = key
            if rep:
                times[p].append(dt * 1e3)
    os.environ.pop("CSA_CHUNK_PLAN", None)
    print(json.dumps({"instance": name, "k": k, "panels": S, "unique": ref[0],
                      "ms": {p: {"best": min(v), "median": statistics.median(v)} for p, v in times.items()},
                      "pair_histogram_materialise_ms": {"best": min(mats) * 1e3,
                                                        "median": statistics.median(mats) * 1e3}}))
