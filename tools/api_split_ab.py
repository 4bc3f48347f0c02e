"""A/B of one legacy_probabilities-sized batch on one GPU (legacy_sample_device, the API's device path):
the one-chunk XT path vs splitting the same panels into chunks drawn on the draw stream while the pair
kernel of the previous chunk runs on the pipeline stream (the XT ring of draw_count_chunks), with the
flat cuts or the round-aligned plan (CSA_CHUNK_PLAN=round: whole rounds of the draw's resident waves, then
one round, then the remainder).  Interleaved calls; best / median wall time; results must agree.
Usage (GPU box): python tools/api_split_ab.py [instance] [k] [S] [reps]"""
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
    import numpy as np
    import torch
    name = sys.argv[1] if len(sys.argv) > 1 else "sf_e_110"
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 110
    S = int(sys.argv[3]) if len(sys.argv) > 3 else 10 ** 6
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    d = os.path.join(REPO, "tests", "golden", "instances", name)
    inst = P.read_instance(os.path.join(d, "categories.csv"), os.path.join(d, "respondents.csv"), k)
    enc = A.encode_cached(inst.categories, inst.agents)
    R = 131072
    variants = {"one": (S, None), "flat_7R": (7 * R, None), "round": (S - 1, "round"), "flat_half": ((S + 1) // 2, None)}
    times = {v: [] for v in variants}
    ref = None
    for rep in range(reps + 1):
        for v, (chunk, plan) in variants.items():
            if plan:
                os.environ["CSA_CHUNK_PLAN"] = plan
            else:
                os.environ.pop("CSA_CHUNK_PLAN", None)
            torch.cuda.synchronize()
            t = time.perf_counter()
            raw = A.legacy_sample_device(enc, k, S, 0, chunk=chunk)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            key = (raw.unique, int(np.asarray(raw.counts).sum()), int(torch.triu(raw.pairs).sum().item()))
            assert ref is None or key == ref, (v, key, ref)
            ref = key
            if rep:
                times[v].append(dt * 1e3)
    os.environ.pop("CSA_CHUNK_PLAN", None)
    print(json.dumps({"instance": name, "k": k, "panels": S, "unique": ref[0],
                      "ms": {v: {"best": round(min(t), 3), "median": round(statistics.median(t), 3)}
                             for v, t in times.items()}}))
