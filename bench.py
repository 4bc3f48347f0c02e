"""LEGACY Monte Carlo benchmark (BASELINE.json metric: panels/s at the sf_e_110 shape).

One "step" = one pass of the hot path (analysis.py:162-191) over one batch of
synthetic-instance panels per GPU, entirely on the device:
draw (with restarts) -> panel hashes -> per-person counts -> pair counts X^T X
(fp4 MFMA) -> distinct-panel count, plus (N > 1) the RCCL exchange (all_reduce of
counts and packed pairs, all_to_all of panel hashes to their owner rank + device
dedupe + all_reduce).  By default step i+1's draw runs on a second stream while
step i is counted (as csa_legacy_sample pipelines its chunks); --no-overlap
serialises them.

    python bench.py [--gpus N --steps K --warmup W] [--config sf_e_110] [--panels P]

Default workload: BASELINE config 2 -- the sf_e_110-shape instance
(tests/golden/instances/sf_e_110, n=1727 k=110 C=7 F=31; synthetic, the real
pool is withheld) at 10^6 panels per GPU per step (weak scaling).  Rank 0
prints ONE JSON line.  The instance and every buffer are resident in HBM
before the timed region.
"""
import argparse
import ctypes
import glob
import importlib
import json
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
PKG = "citizensassemblies-replication_amd"

HBM_PEAK = 8.0e12          # B/s, MI355X spec (MI355X_MICROARCH.md)
I8_MFMA_PEAK = 5.03e15     # dense int8 ops/s: 2x the 2.5 PF bf16 dense rate (MI355X_MICROARCH.md)
FP4_MFMA_PEAK = 10.06e15   # dense fp4 ops/s (scaled f8f6f4 MFMA): 4x the bf16 dense rate (MI355X_MICROARCH.md)
PAIR_ENGINES = {"fp4": (0, FP4_MFMA_PEAK, "fp4 e2m1 operands (exact 0/1 products), f32 accumulation"),
                "i8": (1, I8_MFMA_PEAK, "int8 operands, int32 accumulation")}

CONFIGS = {
    # name: (instance dir, k, default panels per GPU per step)
    "sf_e_110": ("sf_e_110", 110, 10 ** 6),
    "example_large_200": ("example_large_200", 200, 10 ** 6),
    "couples": ("couples_panel_from_twenty_people_no_constraints_2", 2, 10 ** 6),
    "synthetic8192": ("synthetic8192_200", 200, 10 ** 5),
    "example_small_20": ("example_small_20", 20, 10 ** 6),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="sf_e_110", choices=sorted(CONFIGS))
    ap.add_argument("--panels", type=int, default=0, help="panels per GPU per step (0 = config default)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-pairs", action="store_true")
    ap.add_argument("--pair-engine", default="fp4", choices=sorted(PAIR_ENGINES))
    ap.add_argument("--no-overlap", action="store_true",
                    help="run each step's draw after the previous step's counting (default: the draw of step "
                         "i+1 runs on a second stream, into a second panel buffer, while step i is counted)")
    ap.add_argument("--bufs", type=int, default=int(os.environ.get("CSA_BENCH_BUFS", "3")),
                    help="panel buffers in the --overlap pipeline (draw i+1 waits for the counting of step i+1-bufs)")
    ap.add_argument("--count-priority", type=int, default=int(os.environ.get("CSA_BENCH_PRIO", "0")),
                    help="1: the counting stream of the --overlap pipeline is a high-priority stream")
    ap.add_argument("--iso-steps", type=int, default=2,
                    help="serial steps after the timed region that measure each kernel alone (not in `value`)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample duration")
    return ap.parse_args()


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(inst_dir, k, seed, target_s, want_pairs):
    """C oracle (the 'port') on the host cores: draw + counts + pairs + unique on a bounded sample."""
    from oracle import coracle
    from oracle.legacy_oracle import read_instance
    d = os.path.join(REPO, "tests", "golden", "instances", inst_dir)
    o = read_instance(os.path.join(d, "categories.csv"), os.path.join(d, "respondents.csv"), k)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 16))

    def run(S):
        t = time.perf_counter()
        rc, panels, _, _ = coracle.draw(o, k, seed, 0, S, threads=threads)
        assert rc == 0
        coracle.counts(panels, o.n)
        if want_pairs:
            coracle.pairs(panels, o.n, threads=threads)
        coracle.unique(panels, o.n)
        return time.perf_counter() - t

    probe = 2000
    dt = run(probe)
    S = int(min(max(probe, probe * target_s / max(dt, 1e-6)), 5 * 10 ** 6))
    dt = run(S)
    return {"value": S / dt, "unit": "panels/s", "cores": threads, "kind": "port",
            "sample": "%d panels of %s (draw+counts+%sunique), C oracle OpenMP x%d on %s" % (
                S, inst_dir, "pairs+" if want_pairs else "", threads, cpu_model()),
            "seconds": round(dt, 3)}


def load_pmc_traffic(config):
    """HBM bytes per draw launch from a committed rocprofv3 --pmc summary (tools/pmc_summary.py)."""
    path = os.path.join(REPO, "profiles", "pmc_%s.json" % config)
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        return json.load(fh)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print("warning: --gpus %d but WORLD_SIZE %d" % (args.gpus, world), file=sys.stderr)
    # one process per GPU; the modulo only matters for CSA_BENCH_BACKEND=gloo rehearsals of the
    # N > 1 path with several ranks on a 1-GPU box (RCCL refuses two ranks on one device)
    dev_index = local_rank % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = os.environ.get("CSA_BENCH_BACKEND", "nccl")     # nccl = RCCL on ROCm
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    P = importlib.import_module(PKG)
    Dv = importlib.import_module(PKG + ".device")
    Dd = importlib.import_module(PKG + ".distributed")
    inst_dir, k, default_panels = CONFIGS[args.config]
    S = args.panels or default_panels
    d = os.path.join(REPO, "tests", "golden", "instances", inst_dir)
    inst = P.read_instance(os.path.join(d, "categories.csv"), os.path.join(d, "respondents.csv"), k)
    enc = P.encode(inst.categories, inst.agents)
    enc.check_quotas(k)
    want_pairs = not args.no_pairs
    stream = torch.cuda.current_stream(dev)
    if not args.no_overlap and args.count_priority:
        # the counting stream gets the high-priority queue: its workgroups are dispatched ahead of the
        # draw's as draw workgroups retire (the draw holds every VGPR while it runs)
        stream = torch.cuda.Stream(dev, priority=-1)
    engine_id, engine_peak, engine_desc = PAIR_ENGINES[args.pair_engine]
    pipe = Dv.DevicePipeline(enc, k, S, want_pairs=want_pairs, want_unique=True, device=dev, stream=stream,
                             pair_engine=engine_id)
    table = Dd.HashTable(S * world, dev) if world > 1 else None

    draw_name = pipe.draw_kernel_name()   # the kernel csa_draw_async launches (matches rocprofv3 names)
    stages = ["draw", "hash", "xt_count", "pairs", "unique", "exchange"]
    ev_log = []
    last = {"unique": pipe.unique}

    # --overlap (default): step i+1's draw (draw_stream, panel buffer (i+1) % 2) runs while step i is
    # hashed / counted / paired / exchanged on `stream`; every step still does all of its work and
    # the timed region still ends with a device-wide synchronize
    overlap = not args.no_overlap
    draw_stream = torch.cuda.Stream(dev) if overlap else stream
    bufs = [pipe.panels] + [torch.empty_like(pipe.panels) for _ in range(max(args.bufs, 2) - 1)] if overlap \
        else [pipe.panels]
    drawn = [torch.cuda.Event() for _ in bufs]       # draw of the buffer finished (draw_stream)
    counted = [torch.cuda.Event() for _ in bufs]     # counting of the buffer finished (stream)
    with torch.cuda.stream(stream):
        pipe.status.zero_()

    def step(i, log, ov=overlap):
        begin = (i * world + rank) * S            # global panel indices, distinct per step and rank
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(len(stages) + 2)] if log is not None else None
        b = i % len(bufs) if ov else 0
        ds = draw_stream if ov else stream
        pipe.panels = bufs[b]
        if ov:
            ds.wait_event(counted[b])             # step i-2 is done reading this buffer
        if evs:
            evs[-1].record(ds)
        pipe.draw(args.seed, begin, S, stream=ds)
        if evs:
            evs[1].record(ds)
        drawn[b].record(ds)
        stream.wait_event(drawn[b])
        # the pair matrix is not zero-filled: pair_counts stores this step's counts (overwrite), which
        # keeps a 24 MB fill (2.6 ms when it shares the CUs with the next draw) off the counting stream
        pipe.reset(status=False, pairs=False)
        if evs:
            evs[0].record(stream)
        pipe.hash(S)
        if evs:
            evs[2].record(stream)
        pipe.transpose_count(S)
        if evs:
            evs[3].record(stream)
        if want_pairs:
            pipe.pair_counts(S, overwrite=True)
        if evs:
            evs[4].record(stream)
        if world == 1:
            pipe.unique_count(S)
        if evs:
            evs[5].record(stream)
        if world > 1:
            with torch.cuda.stream(stream):   # collectives order on the current stream
                last["unique"] = Dd.combine(pipe.counts, pipe.pairs, pipe.hashes[: 2 * S], table=table,
                                            stream=stream, pair_bound=S * world)[2]
        if evs:
            evs[6].record(stream)
            log.append(evs)
        counted[b].record(stream)

    for i in range(args.warmup):
        step(i, None)
    torch.cuda.synchronize()
    pipe.check_status()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i, ev_log)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    pipe.check_status()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # results of the last timed step (whole job): a rehearsal of --gpus N --panels P must match a
    # single-GPU run with --panels N*P (same global panel indices)
    checks = {"last_step_unique": int(last["unique"].item()), "last_step_count_sum": int(pipe.counts.sum().item()),
              "last_step_pair_sum": int(torch.triu(pipe.pairs.view(enc.n, enc.n)).sum().item()) if want_pairs else None}

    def stage_times(log):
        """per-stage device time (ms) averaged over the logged steps (HIP events on the launch streams)"""
        out = {s: 0.0 for s in stages}
        for evs in log:
            for j, s in enumerate(stages):
                a = evs[-1] if s == "draw" else evs[j] if s != "hash" else evs[0]
                out[s] += a.elapsed_time(evs[j + 1]) / len(log)
        return out

    # stage times inside the timed region; with the two-stream pipeline the counting kernels share
    # the CUs with the next step's draw, so their durations there are inflated.  A short serial pass
    # AFTER the timed region (not part of `value`) measures every kernel alone on the device.
    stage_pipe = stage_times(ev_log)
    iso_log = []
    if overlap:
        torch.cuda.synchronize()
        for i in range(args.iso_steps):
            step(args.warmup + args.steps + i, iso_log, ov=False)
        torch.cuda.synchronize()
        pipe.check_status()
    stage_ms = stage_times(iso_log) if iso_log else stage_pipe
    n, W = enc.n, enc.W
    npad = pipe.npad
    nblk = (S + 63) // 64
    draw_bytes = S * 8 * W                                # packed panel per panel (written once)
    hash_bytes = S * (8 * W + 16)                         # read the panel, write its 128-bit hash
    xt_bytes = S * 8 * W + nblk * npad * 8 + n * 8        # read panels, write transposed bits + counts
    pair_ops = S * n * (n + 1)                            # triangle form of 2*S*n^2
    uniq_bytes = S * (16 + 8 * 2)                         # hashes + table slot traffic (approx.)

    def gbs(b, ms):
        return b / (ms * 1e-3) / 1e9 if ms > 0 else 0.0

    kernels = {
        "draw": {"kernel": draw_name, "ms": stage_ms["draw"],
                 "panels_per_s": S / (stage_ms["draw"] * 1e-3) if stage_ms["draw"] else 0,
                 "bound": "issue (VALU/LDS latency)", "hbm_GBps": gbs(draw_bytes, stage_ms["draw"])},
        "hash": {"kernel": "panel_hash_kernel", "ms": stage_ms["hash"], "hbm_GBps": gbs(hash_bytes, stage_ms["hash"]),
                 "frac": gbs(hash_bytes, stage_ms["hash"]) * 1e9 / HBM_PEAK},
        "xt_count": {"ms": stage_ms["xt_count"], "hbm_GBps": gbs(xt_bytes, stage_ms["xt_count"]),
                     "frac": gbs(xt_bytes, stage_ms["xt_count"]) * 1e9 / HBM_PEAK},
        "unique": {"ms": stage_ms["unique"], "hbm_GBps": gbs(uniq_bytes, stage_ms["unique"])},
    }
    if want_pairs:
        tops = pair_ops / (stage_ms["pairs"] * 1e-3) / 1e12 if stage_ms["pairs"] else 0.0
        kernels["pairs_mfma"] = {"ms": stage_ms["pairs"], "engine": args.pair_engine, "operands": engine_desc,
                                 "TOPs": tops, "ops_per_launch": pair_ops,
                                 "mfma_util": tops * 1e12 / engine_peak, "peak_TOPs": engine_peak / 1e12,
                                 "int8_peak_equiv": tops * 1e12 / I8_MFMA_PEAK,
                                 "note": "ops = S*n*(n+1) (upper triangle incl. diagonal of 2*S*n^2); "
                                         "ms includes the partial-block reduce kernel"}
    if world > 1:
        kernels["exchange"] = {"ms": stage_ms["exchange"]}
    for key, st in (("draw", "draw"), ("hash", "hash"), ("xt_count", "xt_count"), ("unique", "unique"),
                    ("pairs_mfma", "pairs"), ("exchange", "exchange")):
        if key in kernels:
            kernels[key]["ms_in_timed_region"] = stage_pipe[st]
    kernel_timing = ("'ms' = each kernel alone (serial pass of %d steps after the timed region); "
                         "'ms_in_timed_region' = HIP events on the launch streams inside the timed region, "
                         "where the counting kernels share the CUs with the next step's draw" % len(iso_log)
                         ) if iso_log else "HIP events on the launch stream inside the timed region (serial steps)"
    dominant = max(("draw", "hash", "xt_count", "pairs", "unique"), key=lambda s: stage_pipe[s])
    pmc = load_pmc_traffic(args.config)
    # the roofline's kernel duration is the one inside the timed region (what rocprofv3 averages)
    if dominant == "pairs":
        ach = pair_ops / (stage_pipe["pairs"] * 1e-3) / 1e12
        roof = {"kernel": "pair_mfma_kernel", "bound": "mfma", "achieved": ach, "peak": engine_peak / 1e12,
                "unit": "TFLOP/s", "frac": ach * 1e12 / engine_peak, "traffic": None}
    else:
        name = {"draw": draw_name, "hash": "panel_hash_kernel", "xt_count": "xt_count_kernel",
                "unique": "unique_kernel"}[dominant]
        b = {"draw": draw_bytes, "hash": hash_bytes, "xt_count": xt_bytes, "unique": uniq_bytes}[dominant]
        ach = gbs(b, stage_pipe[dominant])
        traffic = None
        pk = (pmc or {}).get("per_kernel", {}).get(name)
        if pk and pmc.get("panels") == S:
            traffic = pk.get("hbm_bytes_per_launch")     # committed rocprofv3 --pmc FETCH/WRITE passes
        roof = {"kernel": name, "bound": "hbm", "achieved": ach, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                "frac": ach * 1e9 / HBM_PEAK, "traffic": traffic}
        if dominant == "draw":
            roof["note"] = ("the draw kernel has no HBM or MFMA roof: it is VALU/LDS issue-bound; 'achieved' is "
                            "its packed-panel writes; issue_frac is the VALU issue-slot fraction from rocprofv3 PMC")
            if pmc and pmc.get("draw_issue") and pmc.get("draw_kernel") == draw_name:
                kernels["draw"]["pmc_issue"] = pmc["draw_issue"]
                roof["issue_frac"] = pmc["draw_issue"].get("valu_issue_frac")

    total = S * world * args.steps
    result = {
        "metric": "LEGACY panels/sec (node) at sf_e_110 shape; XtX MFMA util; speedup vs CPU",
        "value": total / elapsed,
        "unit": "panels/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32/u64 (integer draw), %s MFMA -> exact int pairs" % args.pair_engine,
        "data": "synthetic instance %s (tests/golden/instances), Philox seed %d" % (inst_dir, args.seed),
        "config": {"workload": "%s: %d LEGACY panels/GPU/step, k=%d, n=%d, C=%d, F=%d, counts+%sunique" % (
            args.config, S, k, n, enc.C, enc.F, "pairs+" if want_pairs else ""),
            "panels_per_gpu_per_step": S, "instance": inst_dir, "parallelism": "panel shards x%d" % world,
            "pipeline": ("2 streams: step i+1 drawn while step i is hashed/counted/paired%s" % (
                "/exchanged" if world > 1 else "")) if overlap else "serial"},
        "roofline": roof,
        "kernels": kernels,
        "kernel_timing": kernel_timing,
        "checks": checks,
    }
    if want_pairs:
        result["xtx_mfma_util"] = kernels["pairs_mfma"]["mfma_util"]
        result["xtx_int8_peak_equiv"] = kernels["pairs_mfma"]["int8_peak_equiv"]
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(inst_dir, k, args.seed, args.cpu_seconds, want_pairs)
        result["cpu_baseline"] = cb
        result["speedup_vs_cpu"] = result["value"] / cb["value"]
    elif rank == 0:
        result["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
