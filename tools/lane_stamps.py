"""Segment breakdown of draw_lane_kernel from a CSA_LANE_STAMPS build (diagnostic, GPU box).

    hipcc ... -DCSA_LANE_STAMPS -o exp/libstamps.so csrc/csa_legacy.hip csrc/legacy_mt.cpp
    CSA_LIB=exp/libstamps.so python tools/lane_stamps.py [--config sf_e_110] [--panels 1000000]

Each wave sums s_memtime deltas between four uniform points of its step loop (attempt start +
Philox | the step | cascades | bookkeeping); the totals over all waves give each segment's share
of wave time.  The stamps cost cycles themselves (s_memtime waits on lgkmcnt), so read shares, not
absolute times.
"""
import argparse
import ctypes
import importlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sf_e_110")
    ap.add_argument("--panels", type=int, default=10 ** 6)
    args = ap.parse_args()
    import torch
    import bench
    P = importlib.import_module(bench.PKG)
    N = importlib.import_module(bench.PKG + "._native")
    Dv = importlib.import_module(bench.PKG + ".device")
    inst_dir, k, _ = bench.CONFIGS[args.config]
    d = os.path.join(REPO, "tests", "golden", "instances", inst_dir)
    inst = P.read_instance(os.path.join(d, "categories.csv"), os.path.join(d, "respondents.csv"), k)
    enc = P.encode(inst.categories, inst.agents)
    L = N.lib()
    fn = L.csa_debug_lane_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    out = (ctypes.c_uint64 * 24)()
    S = args.panels
    pipe = Dv.DevicePipeline(enc, k, S, want_pairs=False, want_unique=False)
    pipe.reset()
    for _ in range(2):
        pipe.draw_picks(0, 0, S)
    torch.cuda.synchronize()
    N.check(fn(out, 1))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    pipe.draw_picks(0, S, S)
    ev[1].record()
    torch.cuda.synchronize()
    pipe.check_status()
    N.check(fn(out, 1))
    names = ["attempt starts + Philox", "step (argmax, scan, select, decrements)", "cascades", "bookkeeping + loop"]
    tot = max(1, sum(out[q] for q in range(4)))
    waves = out[8]
    res = {"config": args.config, "panels": S, "kernel": pipe.draw_kernel_name(), "ms": ev[0].elapsed_time(ev[1]),
           "waves": waves, "cycles_per_wave": tot / max(waves, 1),
           "share": {names[q]: out[q] / tot for q in range(4)},
           "cycles_per_wave_by_segment": {names[q]: out[q] / max(waves, 1) for q in range(4)},
           # region execution counts per wave (tools/valu_budget.py multiplies them with the regions'
           # static VALU classes)
           "region_runs_per_wave": {r: out[9 + q] / max(waves, 1) for q, r in enumerate(
               ("loop", "philox", "step", "pick", "store", "round", "pass2", "pass1", "nocand", "kcheck",
                "ending"))}}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
