"""One GPU's share of BASELINE configs 3 and 5, end to end through the Python API (timed, with the
results' invariants checked): legacy_probabilities(example_large_200, S) and (synthetic8192, S).
Prints one JSON line.  Usage (GPU box): python tools/scale_runs.py [S_large] [S_synthetic]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import importlib  # noqa: E402

P = importlib.import_module("citizensassemblies-replication_amd")
A = importlib.import_module("citizensassemblies-replication_amd.analysis")


def run(name, k, S):
    d = os.path.join(REPO, "tests", "golden", "instances", name)
    inst = P.read_instance(os.path.join(d, "categories.csv"), os.path.join(d, "respondents.csv"), k)
    A.legacy_probabilities(inst, 1000, 0, keep_panels=False)           # warm: encoding + pipeline
    import torch
    torch.cuda.synchronize()
    t = time.perf_counter()
    alloc, found, hist = A.legacy_probabilities(inst, S, 0, keep_panels=False)
    dt = time.perf_counter() - t
    total = sum(alloc.values())
    assert abs(total - k) < 1e-6 * k, total                            # sum of probabilities = k
    return {"instance": name, "k": k, "panels": S, "seconds": round(dt, 4), "panels_per_s": S / dt,
            "unique": len(found), "sum_alloc": total}


if __name__ == "__main__":
    s1 = int(sys.argv[1]) if len(sys.argv) > 1 else 1250000
    s2 = int(sys.argv[2]) if len(sys.argv) > 2 else 12500000
    out = {"note": "one MI355X's share of BASELINE config 3 (10^7 example_large_200 panels / 8 GPUs) and "
                   "config 5 (10^8 synthetic n=8192 panels / 8 GPUs) through legacy_probabilities "
                   "(counts, pairs and the exact distinct count on the device; the pair histogram stays "
                   "on the device until read)",
           "config3_share": run("example_large_200", 200, s1),
           "config3_whole_on_one_gpu": run("example_large_200", 200, 8 * s1),
           "config5_share": run("synthetic8192_200", 200, s2)}
    print(json.dumps(out))
