"""Bit transpose + counts microbenchmark on the GPU box: csa_transpose_count_async (xt_count_kernel) on
random packed panels alone, timed with HIP events on the launch stream, for several pool sizes.  Bytes =
the algorithmic 8 W B read + 8 npad / 64 B written per panel.  CSA_XT_KERNEL selected variants in
round 4 (profiles/r04_xt_ab/); --variants keeps that interface for a library that has them.

    python tools/xt_bench.py [--n 1727,2000,200,8192] [--panels 1000000] [--reps 10]
"""
import argparse
import ctypes
import importlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="1727,2000,200,8192")
    ap.add_argument("--panels", type=int, default=10 ** 6)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default="default")
    args = ap.parse_args()
    import torch
    N = importlib.import_module("citizensassemblies-replication_amd._native")
    L = N.lib()
    S = args.panels
    stream = torch.cuda.current_stream()
    res = []
    for n in (int(x) for x in args.n.split(",")):
        W = (n + 63) // 64
        npad = int(L.csa_xt_pad(n))
        nblk = (S + 63) // 64
        g = torch.Generator(device="cuda").manual_seed(n)
        p = torch.randint(-2 ** 63, 2 ** 63 - 1, (S, W), device="cuda", generator=g)
        p &= torch.randint(-2 ** 63, 2 ** 63 - 1, (S, W), device="cuda", generator=g)
        if n % 64:
            p[:, -1] &= (1 << (n % 64)) - 1
        nbytes = S * 8 * W + nblk * 8 * npad
        ref = None
        for var in args.variants.split(","):
            if var != "default":
                os.environ["CSA_XT_KERNEL"] = var
            xt = torch.empty(nblk * npad, dtype=torch.int64, device="cuda")
            cnt = torch.zeros(n, dtype=torch.int64, device="cuda")
            times = []
            for r in range(args.reps + 1):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                N.check(L.csa_transpose_count_async(N.ptr(p), S, n, N.ptr(xt), N.ptr(cnt),
                                                    ctypes.c_void_p(stream.cuda_stream)))
                e1.record(stream)
                torch.cuda.synchronize()
                if r:
                    times.append(e0.elapsed_time(e1))
            got = (xt.clone(), cnt // (args.reps + 1))
            same = True if ref is None else bool(torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]))
            ref = got if ref is None else ref
            ms = min(times)
            row = {"n": n, "W": W, "panels": S, "variant": var, "ms": ms, "ms_median": sorted(times)[len(times) // 2],
                   "bytes": nbytes, "TBps": nbytes / (ms * 1e-3) / 1e12, "equal_to_first": same}
            res.append(row)
            print(json.dumps(row), flush=True)
    os.environ.pop("CSA_XT_KERNEL", None)


if __name__ == "__main__":
    main()
