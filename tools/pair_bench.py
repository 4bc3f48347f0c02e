"""X^T X microbenchmark on the GPU box: csa_pair_counts_ex_async on random transposed bits (plane
layout, ~2.5 % density like k = 200 of n = 8192) for each kernel variant (CSA_PAIR_KERNEL), timed
with HIP events on the launch stream; every variant's pair counts must equal the first one's.

    python tools/pair_bench.py [--n 8192] [--panels 1000000] [--reps 5] [--variants tile,split]
"""
import argparse
import importlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--panels", type=int, default=10 ** 6)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default="tile4,tile2,split")
    ap.add_argument("--engine", default="fp4", choices=("fp4", "i8"))
    ap.add_argument("--density", type=float, default=0.025)
    args = ap.parse_args()
    import torch
    N = importlib.import_module("citizensassemblies-replication_amd._native")
    L = N.lib()
    n, S = args.n, args.panels
    npad = int(L.csa_xt_pad(n))
    nblk = (S + 63) // 64
    g = torch.Generator(device="cuda").manual_seed(1)
    # random words with ~density ones: AND of log2(1/density) random words
    ands = max(1, round(-torch.log2(torch.tensor(args.density)).item()))
    xt = torch.randint(-2 ** 63, 2 ** 63 - 1, (nblk * npad,), device="cuda", generator=g)
    for _ in range(ands - 1):
        xt &= torch.randint(-2 ** 63, 2 ** 63 - 1, (nblk * npad,), device="cuda", generator=g)
    xt = xt.view(nblk, npad)
    xt[:, n:] = 0
    engine = {"fp4": N.CSA_PAIR_FP4, "i8": N.CSA_PAIR_I8}[args.engine] | N.CSA_PAIR_OVERWRITE
    ops = S * n * (n + 1)
    peak = 10.06e15 if args.engine == "fp4" else 5.03e15
    stream = torch.cuda.current_stream()
    out, ref = {}, None
    for var in args.variants.split(","):
        # split = pair_mfma_kernel; tile<NB> = pair_fp4_tile_kernel<NB> (CSA_P2_NB); tile = the default
        os.environ["CSA_PAIR_KERNEL"] = "1" if var == "split" else "2"
        os.environ.pop("CSA_P2_NB", None)
        if var.startswith("tile") and len(var) > 4:
            os.environ["CSA_P2_NB"] = var[4:]
        sb = int(L.csa_pair_scratch_bytes(n, nblk, engine))
        scr = torch.empty(max(sb, 4) // 4 + 1, dtype=torch.int32, device="cuda")
        pairs = torch.zeros(n * n, dtype=torch.int64, device="cuda")
        times = []
        for r in range(args.reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            N.check(L.csa_pair_counts_ex_async(N.ptr(xt), nblk, n, N.ptr(pairs), engine, N.ptr(scr), sb,
                                               ctypes_stream(stream)))
            e1.record(stream)
            torch.cuda.synchronize()
            if r:
                times.append(e0.elapsed_time(e1))
        up = torch.triu(pairs.view(n, n))
        same = True if ref is None else bool(torch.equal(up, ref))
        ref = up if ref is None else ref
        ms = min(times)
        out[var] = {"ms": ms, "ms_all": times, "TOPs": ops / (ms * 1e-3) / 1e12, "frac": ops / (ms * 1e-3) / peak,
                    "equal_to_first": same, "scratch_MB": sb / 1e6}
        print(var, json.dumps(out[var]), flush=True)
    print(json.dumps({"n": n, "panels": S, "engine": args.engine, "ops": ops, "variants": out}))


def ctypes_stream(stream):
    import ctypes
    return ctypes.c_void_p(stream.cuda_stream)


if __name__ == "__main__":
    main()
