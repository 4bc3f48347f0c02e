"""Measure the SURVEY.md section 8(f) rows on one GPU; prints one JSON object.

  f1  xmin._get_panel_not_in_portfolio_if_possible (xmin.py:464-474): device call latency vs
      the same legacy_find calls in the C oracle (1 core)
  f2  cache.run_legacy_or_retrieve npz write / read at sf_e, 10^6 panels
  f3  pair_histogram_kernel (sorted pair-probability curve, analysis.py:339-342): kernel time and
      HBM GB/s over the upper triangle at sf_e (n=1727) and n=8192, vs numpy sort of the triangle

    python tools/bench_rows.py [--panels 1000000]
"""
import argparse
import ctypes
import importlib
import json
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "citizensassemblies-replication_amd"
INST = os.path.join(REPO, "tests", "golden", "instances")


def paths(name):
    return os.path.join(INST, name, "categories.csv"), os.path.join(INST, name, "respondents.csv")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--panels", type=int, default=10 ** 6)
    args = ap.parse_args()
    import torch
    P = importlib.import_module(PKG)
    X = importlib.import_module(PKG + ".xmin")
    Cc = importlib.import_module(PKG + ".cache")
    St = importlib.import_module(PKG + ".stats")
    Dv = importlib.import_module(PKG + ".device")
    N = importlib.import_module(PKG + "._native")
    from oracle import coracle
    from oracle.legacy_oracle import read_instance as oread
    out = {}

    # ---- f1 -------------------------------------------------------------------------------
    inst = P.read_instance(*paths("sf_e_110"), 110)
    enc = P.encode(inst.categories, inst.agents)
    o = oread(*paths("sf_e_110"), 110)
    _, head, _, _ = coracle.draw(o, 110, 0, 0, 40)
    portfolio = [frozenset(enc.agent_ids[p] for p in P.instance.unpack_panel(r, enc.n)) for r in head]
    X._get_panel_not_in_portfolio_if_possible(inst.categories, inst.agents, 110, portfolio)   # warm-up
    reps = 20
    t = time.perf_counter()
    for _ in range(reps):
        P.seed(0)
        X._get_panel_not_in_portfolio_if_possible(inst.categories, inst.agents, 110, portfolio)
    dev_s = (time.perf_counter() - t) / reps
    t = time.perf_counter()
    coracle.draw(o, 110, 0, 0, 41, threads=1)
    cpu_s = time.perf_counter() - t
    out["f1_xmin_caller"] = {"instance": "sf_e_110", "portfolio": len(portfolio), "first_non_member": 40,
                             "device_ms_per_call": dev_s * 1e3, "c_oracle_1core_ms_same_41_draws": cpu_s * 1e3,
                             "reference_python_ms_est": 41 * 1e3 / 30.2,
                             "note": "device call includes encode, portfolio upload + hash table, chunked draws"}

    # ---- f2 -------------------------------------------------------------------------------
    S = args.panels
    with tempfile.TemporaryDirectory() as d:
        t = time.perf_counter()
        Cc.run_legacy_or_retrieve("sf_e_110", inst, False, directory=d, iterations=S, keep_panels=False)
        first = time.perf_counter() - t
        f = Cc.legacy_cache_path("sf_e_110", 110, False, d)
        size = os.path.getsize(f)
        t = time.perf_counter()
        _, _, hist = Cc.run_legacy_or_retrieve("sf_e_110", inst, False, directory=d, iterations=S, keep_panels=False)
        second = time.perf_counter() - t
    out["f2_cache"] = {"instance": "sf_e_110", "panels": S, "compute_and_write_s": first, "read_s": second,
                       "npz_bytes": size, "pair_entries": enc.n * (enc.n - 1) // 2}

    # ---- f3 -------------------------------------------------------------------------------
    f3 = {}
    for name, k, S3 in [("sf_e_110", 110, S), ("synthetic8192_200", 200, 20000)]:
        inst3 = P.read_instance(*paths(name), k)
        enc3 = P.encode(inst3.categories, inst3.agents)
        pipe = Dv.DevicePipeline(enc3, k, S3, want_unique=False)
        pipe.reset()
        pipe.run(0, 0, S3)
        pipe.check_status()
        n = enc3.n
        n_bins = int(pipe.counts.max().item()) + 1
        hist = torch.empty(n_bins, dtype=torch.int64, device="cuda")
        over = torch.empty(1, dtype=torch.int64, device="cuda")
        st = torch.cuda.current_stream()
        for _ in range(3):
            N.check(N.lib().csa_pair_histogram_async(N.ptr(pipe.pairs), n, N.ptr(hist), n_bins, N.ptr(over),
                                                     ctypes.c_void_p(st.cuda_stream)))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record(st)
        for _ in range(reps):
            N.check(N.lib().csa_pair_histogram_async(N.ptr(pipe.pairs), n, N.ptr(hist), n_bins, N.ptr(over),
                                                     ctypes.c_void_p(st.cuda_stream)))
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        tri = n * (n - 1) // 2
        m = pipe.pairs.view(n, n).cpu().numpy()
        t = time.perf_counter()
        np.sort(m[np.triu_indices(n, 1)])
        np_s = time.perf_counter() - t
        f3[name] = {"n": n, "panels": S3, "bins": n_bins, "kernel_ms": ms, "bytes": tri * 8,
                    "hbm_GBps": tri * 8 / (ms * 1e-3) / 1e9, "numpy_sort_ms": np_s * 1e3,
                    "note": "kernel_ms includes the two memsets of the histogram"}
    out["f3_pair_histogram"] = f3
    print(json.dumps(out))


if __name__ == "__main__":
    main()
