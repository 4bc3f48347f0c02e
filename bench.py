"""LEGACY Monte Carlo benchmark (BASELINE.json metric: panels/s at the sf_e_110 shape).

One "step" = one pass of the hot path (analysis.py:162-191) over one batch of
synthetic-instance panels per GPU, entirely on the device:
draw (with restarts; pick lists) -> pack (packed panels + 128-bit hashes) ->
bit transpose + per-person counts -> pair counts X^T X (fp4 MFMA) -> exact
distinct-panel count, plus (N > 1) the exchange (RCCL all_reduce of counts and
packed pairs, equal-split all_to_alls of the local distinct panels to their
owner ranks + exact owner dedupe + all_reduce; nothing in it waits on the host).
The draws run on their own stream, enqueued --bufs - 1 steps ahead of the
counting; --no-overlap serialises everything on one stream.

    python bench.py [--gpus N --steps K --warmup W] [--config sf_e_110] [--panels P]

Default workload: BASELINE config 2 -- the sf_e_110-shape instance
(tests/golden/instances/sf_e_110, n=1727 k=110 C=7 F=31; synthetic, the real
pool is withheld) at 10^6 panels per GPU per step (weak scaling), 400 timed
steps (~2 s).  Rank 0 prints ONE JSON line.  The instance and every buffer are
resident in HBM before the timed region.
"""
import argparse
import glob
import hashlib
import importlib
import json
import os
import platform
import subprocess
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
    "synthetic8192": ("synthetic8192_200", 200, 10 ** 6),   # 10^5 per step left 3.05 rounds of waves: 17.8 vs 18.4 M/s
    "example_small_20": ("example_small_20", 20, 10 ** 6),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="sf_e_110", choices=sorted(CONFIGS))
    ap.add_argument("--panels", type=int, default=0, help="panels per GPU per step (0 = config default)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-pairs", action="store_true")
    ap.add_argument("--pair-engine", default="fp4", choices=sorted(PAIR_ENGINES))
    ap.add_argument("--no-overlap", action="store_true",
                    help="serialise every stage on one stream (default: draws on their own stream, "
                         "--bufs - 1 steps ahead of the counting)")
    ap.add_argument("--bufs", type=int, default=3, help="panel buffers of the draw/count pipeline")
    ap.add_argument("--count-priority", type=int, default=int(os.environ.get("CSA_COUNT_PRIORITY", "0")),
                    help="1: counting stream at the highest stream priority (A/B)")
    ap.add_argument("--draw-streams", type=int, default=int(os.environ.get("CSA_DRAW_STREAMS", "1")),
                    help="streams the draws of consecutive steps alternate over (A/B only: > 1 needs a library "
                         "with a pick-list ring, profiles/r04f_draw_streams/, and measured slower)")
    ap.add_argument("--pack-on", default="fused", choices=("fused", "draw", "count"),
                    help="where pick lists become panels: inside the draw kernel (fused, default), "
                         "picks_pack_kernel after the draw on the draw stream, or first on the counting "
                         "stream (one pick-list buffer per panel buffer)")
    ap.add_argument("--xt-from", default="draw", choices=("draw", "count"),
                    help="where the pair kernel's XT operand comes from: the draw kernel's fused pack "
                         "(csa_draw_xt_async, one XT buffer per panel buffer; the counts are then the pair "
                         "matrix's diagonal) where the instance's draw kernel has one, else -- or with "
                         "'count' -- xt_count_kernel on the counting stream")
    ap.add_argument("--iso-steps", type=int, default=2,
                    help="serial steps after the timed region that measure each kernel alone (not in `value`)")
    ap.add_argument("--exchange", default="keys", choices=("keys", "bitmask"),
                    help="N > 1: distinct panels travel as 24-byte keys (default) or with their bitmasks")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target duration of each CPU-baseline leg")
    ap.add_argument("--no-api", action="store_true", help="skip the legacy_probabilities end-to-end leg")
    ap.add_argument("--job-panels", type=int, default=0,
                    help="strong scaling (BASELINE configs 3 and 5): time ONE job of this many panels split "
                         "over the N ranks (each rank's share in chunks of --panels; counts and pairs "
                         "accumulated over the job, the exact distinct count over all of its panels); "
                         "--steps is ignored, --warmup chunks of a throwaway job run first")
    return ap.parse_args()


def digests(counts, pairs, n):
    """SHA-256 of the final per-person count vector (int64, little-endian) and of the pair matrix's
    upper triangle incl. the diagonal (np.triu of the int64 n x n matrix): equal digests at N = 1 and
    N > 1 mean the whole vectors are equal, not just their sums."""
    import numpy as np
    out = {"counts_sha256": hashlib.sha256(np.ascontiguousarray(counts.cpu().numpy(), "<i8").tobytes()).hexdigest()}
    if pairs is not None:
        m = pairs.view(n, n).cpu().numpy()
        out["pairs_triu_sha256"] = hashlib.sha256(np.ascontiguousarray(np.triu(m), "<i8").tobytes()).hexdigest()
    return out


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_quota():
    """CPUs the cgroup lets this process use (cpu.max), or None when unlimited / unknown."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, p = fh.read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def source_sha():
    """Digest of the kernel sources: a committed PMC profile is only used for the same kernels."""
    h = hashlib.sha256()
    for path in sorted(glob.glob(os.path.join(REPO, PKG, "csrc", "*"))):
        with open(path, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


_PY_LEG = r"""
import json, sys, time
sys.path.insert(0, %(repo)r)
from oracle.legacy_oracle import read_instance, legacy_probabilities
o = read_instance(%(cat)r, %(resp)r, %(k)d)
t = time.perf_counter()
r = legacy_probabilities(o, %(S)d, %(seed)d, panel_begin=%(begin)d)
print(json.dumps({"seconds": time.perf_counter() - t, "unique": r.unique}))
"""


def python_leg(d, k, seed, S, procs):
    """The Python restatement of the reference loop (oracle/legacy_oracle.py: draws, Counter, pair
    counts, distinct set) in `procs` single-threaded processes of S panels each, started together."""
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    cat, resp = os.path.join(d, "categories.csv"), os.path.join(d, "respondents.csv")
    t = time.perf_counter()
    ps = [subprocess.Popen([sys.executable, "-c", _PY_LEG % dict(repo=REPO, cat=cat, resp=resp, k=k, S=S, seed=seed,
                                                                 begin=j * S)],
                           env=env, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL) for j in range(procs)]
    outs = [p.communicate()[0] for p in ps]
    wall = time.perf_counter() - t
    if any(p.returncode for p in ps):
        raise RuntimeError("python CPU-baseline leg failed")
    inner = max(json.loads(o)["seconds"] for o in outs)
    return procs * S / wall, wall, inner


def cpu_baseline(inst_dir, k, seed, target_s, want_pairs):
    """CPU legs on this host, bounded samples of the same workload:
    the C OpenMP port on every host core (`value`, `cores`), the Python restatement of the
    reference loop on one core, and one Python process per host core."""
    from oracle import coracle
    from oracle.legacy_oracle import read_instance
    d = os.path.join(REPO, "tests", "golden", "instances", inst_dir)
    o = read_instance(os.path.join(d, "categories.csv"), os.path.join(d, "respondents.csv"), k)
    visible = len(os.sched_getaffinity(0))
    quota = cpu_quota()
    # the CPU time this process may use: every visible core unless the cgroup caps it (cpu.max)
    usable = max(1, min(visible, int(quota))) if quota else visible

    def run(S, threads):
        t = time.perf_counter()
        rc, panels, _, _ = coracle.draw(o, k, seed, 0, S, threads=threads)
        assert rc == 0
        coracle.counts(panels, o.n)
        if want_pairs:
            coracle.pairs(panels, o.n, threads=threads)
        coracle.unique(panels, o.n)
        return time.perf_counter() - t

    legs = {}
    for threads in sorted({visible, usable}):
        probe = 4000
        dt = run(probe, threads)
        S = int(min(max(probe, probe * target_s / max(dt, 1e-6)), 10 ** 7))
        dt = run(S, threads)
        legs[threads] = (S / dt, S, dt)
    best = max(legs, key=lambda t: legs[t][0])
    rate, S, dt = legs[best]
    out = {"value": rate, "unit": "panels/s", "cores": best, "kind": "port",
           "sample": "%d panels of %s (draw+counts+%sunique), C oracle OpenMP x%d threads on %s" % (
               S, inst_dir, "pairs+" if want_pairs else "", best, cpu_model()),
           "seconds": round(dt, 3), "cpu_model": cpu_model(), "host_cpus_visible": visible,
           "cgroup_cpu_quota": quota,
           "port_by_threads": {str(t): {"panels_per_s": v[0], "panels": v[1], "seconds": round(v[2], 3)}
                               for t, v in legs.items()},
           "cores_note": "every visible host core was tried; the box's cgroup grants %s CPUs of time "
                         "(cpu.max), so `cores` is the thread count that ran fastest" % quota}
    # Python restatement: probe, then ~target_s per process
    rate1, w1, _ = python_leg(d, k, seed, 20, 1)
    S1 = max(20, int(rate1 * target_s * 0.8))
    rate1, w1, _ = python_leg(d, k, seed, S1, 1)
    out["python_1core"] = {"value": rate1, "unit": "panels/s", "cores": 1, "panels": S1, "seconds": round(w1, 3),
                           "sample": "oracle/legacy_oracle.py (Python restatement of analysis.py:162-191), 1 process"}
    Sp = max(10, int(rate1 * target_s * 0.5))
    ratep, wp, innerp = python_leg(d, k, seed, Sp, usable)
    out["python_per_core"] = {"value": ratep, "unit": "panels/s", "cores": usable, "panels_per_process": Sp,
                              "seconds": round(wp, 3), "slowest_process_seconds": round(innerp, 3),
                              "sample": "%d single-threaded Python processes (one per usable host core) of %d "
                                        "panels" % (usable, Sp)}
    out["reference_python_note"] = ("the unmodified reference (Python, dict + deepcopy) ran at 30.2 panels/s on one "
                                    "core at this shape (SURVEY.md section 6, dev container)")
    return out


def load_valu_budget(config):
    """Class-weighted VALU budget of the draw kernel (tools/valu_budget.py, profiles/valu_budget_<config>.json):
    its dynamic VALU mix split into the two issue classes measured by tools/coissue.hip -- two-operand
    add/and/or/xor/mov/lshr with VGPR or constant operands, which two waves of a SIMD issue together
    (2.47 SIMD cycles each), and everything else (bcnt, cndmask, mul24, 3-source ops, DPP, SDWA, an SGPR
    operand: one per ~4.3 cycles) -- priced per panel.  That budget is the kernel's VALU roof."""
    path = os.path.join(REPO, "profiles", "valu_budget_%s.json" % config)
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        return json.load(fh)


def load_pmc(config):
    """Committed rocprofv3 --pmc summary (tools/make_pmc_profile.py) for this config."""
    path = os.path.join(REPO, "profiles", "pmc_%s.json" % config)
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        return json.load(fh)


def api_leg(P, A, inst, S, seed):
    """legacy_probabilities(instance, S, seed) end to end (analysis.py:162 signature): first call,
    then the steady state (cached encoding + device pipeline), then the host materialisation of the
    n*n pair histogram and of the per-person dict."""
    import torch
    t = time.perf_counter()
    A.legacy_probabilities(inst, S, seed)
    first = time.perf_counter() - t
    runs, mats = [], []
    for _ in range(10):
        torch.cuda.synchronize()
        t = time.perf_counter()
        alloc, found, hist = A.legacy_probabilities(inst, S, seed)
        runs.append(time.perf_counter() - t)
        t = time.perf_counter()
        hist.upper()
        mats.append(time.perf_counter() - t)
    srt = sorted(runs)
    return {"call": "legacy_probabilities(sf_e_110 instance, %d, %d)" % (S, seed), "first_call_ms": first * 1e3,
            "ms": srt[0] * 1e3, "ms_median": srt[len(srt) // 2] * 1e3, "ms_runs": [r * 1e3 for r in runs],
            "pair_histogram_materialise_ms": min(mats) * 1e3, "pair_histogram_materialise_first_ms": mats[0] * 1e3,
            "unique": len(found), "note": "returns the alloc dict, the exact distinct count (found_panels decodes "
                                          "the device panels when iterated) and a PairHistogram whose strict upper "
                                          "triangle is packed and divided by S on the device and copied on first "
                                          "access (pair_histogram_materialise_ms: best of 10 calls; _first_ms "
                                          "includes the process's first pinned host allocation)"}


def self_launch(n, script=None, argv=None, grace=10.0):
    """`python bench.py --gpus N` without a launcher: start N rank processes of this same command
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, one GPU each) and return the worst exit code.
    Runs before anything imports torch or touches a device in this process.  The ranks are polled:
    when one exits non-zero the others (otherwise blocked in a rendezvous or collective until its
    timeout) are terminated, then killed after ``grace`` seconds, and that first exit code returned."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] +
                                      list(sys.argv[1:] if argv is None else argv), env=env))
    first_bad = 0
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc]
        if bad:
            first_bad = bad[0]
            break
        if all(rc is not None for rc in rcs):
            return 0
        time.sleep(0.05)
    for p in procs:               # a rank failed: the others would wait for it until their timeout
        if p.poll() is None:
            p.terminate()
    deadline = time.time() + grace
    for p in procs:
        try:
            p.wait(timeout=max(0.0, deadline - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    return first_bad


def run_job(args, world, rank, dev, torch, dist, A, Dd, enc, k, S, inst_dir, pipe, want_pairs, stream, draw_name):
    """--job-panels P: one whole job of P panels (global indices 0 .. P-1) split over the ranks in
    contiguous shares (distributed.shard_range), every rank's share drawn in chunks of S panels.  All
    draws are enqueued on the draw stream at once (each chunk has its own slice of the share's panel
    buffer, so nothing waits for the counting), the counting stream follows chunk by chunk (counts and
    pairs accumulate over the job), then the exact distinct count over the whole share (N = 1) or the
    exchange of section 5 (N > 1: all_reduce of counts and packed pairs, 24-byte keys to the owners).
    value = P / (the max over ranks of the barrier-to-barrier time of the whole job)."""
    import ctypes
    N = importlib.import_module(PKG + "._native")
    Pj = int(args.job_panels)
    b0, e0 = Dd.shard_range(Pj, world, rank)
    share, n_max = e0 - b0, Dd.shard_range(Pj, world, 0)[1]
    W = enc.W
    draw_streams = [torch.cuda.Stream(dev) for _ in range(max(args.draw_streams, 1))]
    panels_all = torch.empty(max(share * W, 1), dtype=torch.int64, device=dev)
    hashes_all = torch.empty(max(2 * share, 2), dtype=torch.int64, device=dev)
    table = Dd.HashTable(max(share, 1), dev) if world == 1 else None
    xchg = Dd.PanelExchange(n_max, W, world, dev, redraw=(enc.handle, k, args.seed, 0)
                            if args.exchange == "keys" else None) if world > 1 else None

    # XT from the draw's fused pack (as the weak-scaling step): a ring of XT buffers, the draw of chunk j
    # waiting for the pairs of chunk j - ring (long done), the counts the pair diagonal at the end
    xt_draw = want_pairs and args.xt_from == "draw" and args.draw_streams == 1 and pipe.xt_fused()
    xring = [pipe.xt] + [torch.empty_like(pipe.xt) for _ in range(2)] if xt_draw else None

    def job(begin, count):
        steps = (count + S - 1) // S
        with torch.cuda.stream(stream):
            pipe.status.zero_()
            pipe.counts.zero_()
            if want_pairs and count == 0:
                pipe.pairs.zero_()
        if xt_draw and steps:
            drawn, counted = [], []

            def count_chunk(j):
                o, ln = j * S, min(S, count - j * S)
                stream.wait_event(drawn[j])
                pipe.xt = xring[j % len(xring)]
                pipe.pair_counts(ln, overwrite=j == 0, shared=j + 1 < steps)
                ev = torch.cuda.Event()
                ev.record(stream)
                counted.append(ev)

            ds = draw_streams[0]
            for j in range(steps):
                o, ln = j * S, min(S, count - j * S)
                if j >= len(xring):
                    ds.wait_event(counted[j - len(xring)])
                pipe.panels, pipe.hashes = panels_all[o * W:(o + ln) * W], hashes_all[2 * o:2 * (o + ln)]
                pipe.xt = xring[j % len(xring)]
                assert pipe.draw_xt(args.seed, begin + o, ln, stream=ds)
                ev = torch.cuda.Event()
                ev.record(ds)
                drawn.append(ev)
                if j:
                    count_chunk(j - 1)
            count_chunk(steps - 1)
            pipe.counts_from_pairs()
            pipe.xt = xring[0]
        drawn = []
        for j in range(0 if xt_draw else steps):
            o, ln = j * S, min(S, count - j * S)
            pipe.panels, pipe.hashes = panels_all[o * W:(o + ln) * W], hashes_all[2 * o:2 * (o + ln)]
            ds = draw_streams[j % len(draw_streams)]
            pipe.draw(args.seed, begin + o, ln, stream=ds)
            ev = torch.cuda.Event()
            ev.record(ds)
            drawn.append(ev)
        for j in range(0 if xt_draw else steps):
            o, ln = j * S, min(S, count - j * S)
            stream.wait_event(drawn[j])
            pipe.panels, pipe.hashes = panels_all[o * W:(o + ln) * W], hashes_all[2 * o:2 * (o + ln)]
            pipe.transpose_count(ln)
            if want_pairs:
                pipe.pair_counts(ln, overwrite=j == 0, shared=j + 1 < steps)
        if world == 1:
            table.ensure(count)
            with torch.cuda.stream(stream):
                table.count.zero_()
            N.check(N.lib().csa_unique_async(N.ptr(hashes_all), N.ptr(panels_all), count, W, N.ptr(table.table),
                                             table.slots, N.ptr(table.count), N.ptr(pipe.status),
                                             ctypes.c_void_p(stream.cuda_stream)))
            return table.count, steps
        with torch.cuda.stream(stream):
            _, _, u = Dd.combine(pipe.counts, pipe.pairs if want_pairs else None, hashes_all[: 2 * count],
                                 panels_all[: count * W], W, exchange=xchg, stream=stream, pair_bound=Pj,
                                 status=pipe.status, panel_begin=begin)
        return u, steps

    # warmup: a throwaway job of --warmup chunks on this rank's first panels
    job(b0, min(share, args.warmup * S))
    torch.cuda.synchronize()
    pipe.check_status()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    A.draw_stats(enc, reset=True)
    t0 = time.perf_counter()
    u, steps = job(b0, share)
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
        st = torch.tensor([steps], dtype=torch.int64, device=dev)
        dist.all_reduce(st, op=dist.ReduceOp.MAX)
        steps = int(st.item())
    checks = {"job_unique": int(u.item()), "job_count_sum": int(pipe.counts.sum().item()),
              "job_pair_sum": int(torch.triu(pipe.pairs.view(enc.n, enc.n)).sum().item()) if want_pairs else None}
    checks.update({"job_" + key: v for key, v in digests(pipe.counts, pipe.pairs if want_pairs else None,
                                                       enc.n).items()})
    stt = torch.tensor(list(A.draw_stats(enc).values()), dtype=torch.int64, device=dev)
    if world > 1:
        Dd._all_reduce(stt)
    draw_stats = dict(zip(A.STAT_KEYS, (int(x) for x in stt.cpu().tolist())))
    draw_stats["panels"] = Pj
    result = {
        "metric": "LEGACY panels/sec (node) at sf_e_110 shape; XtX MFMA util; speedup vs CPU",
        "value": Pj / elapsed,
        "unit": "panels/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / max(steps, 1) * 1e3,
        "job_seconds": elapsed,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int32/u64 (integer draw), %s MFMA -> exact int pairs" % args.pair_engine,
        "data": "synthetic instance %s (tests/golden/instances), Philox seed %d" % (inst_dir, args.seed),
        "config": {"workload": "%s: ONE job of %d LEGACY panels over %d GPU(s) (shares of <= %d, chunks of %d), "
                               "k=%d, n=%d, counts+%sunique over the whole job" % (
                                   args.config, Pj, world, n_max, S, k, enc.n, "pairs+" if want_pairs else ""),
                   "job_panels": Pj, "chunk_panels": S, "instance": inst_dir,
                   "parallelism": "panel shards x%d" % world, "draw_kernel": draw_name,
                   "pipeline": ("chunk draws on the draw stream, each writing its XT operand (3-buffer ring); the "
                                "pair kernel follows per chunk, the counts are the pair diagonal") if xt_draw else
                               "every chunk's draw enqueued at once on the draw stream; counting follows per chunk"},
        "checks": checks,
        "draw_stats": draw_stats,
        "cpu_baseline": None,
    }
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%d (launch with matching --nproc-per-node, or without a "
                 "launcher: bench.py starts --gpus ranks itself)" % (args.gpus, world))
    import torch
    import torch.distributed as dist
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
    A = importlib.import_module(PKG + ".analysis")
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
    if args.count_priority:
        # the counting / exchange stream at the highest priority: its workgroups dispatch before the
        # draws' when both wait for CU slots (A/B with --draw-streams > 1)
        stream = torch.cuda.Stream(dev, priority=torch.cuda.Stream.priority_range()[1])
    engine_id, engine_peak, engine_desc = PAIR_ENGINES[args.pair_engine]
    pipe = Dv.DevicePipeline(enc, k, S, want_pairs=want_pairs, want_unique=True, device=dev, stream=stream,
                             pair_engine=engine_id)
    draw_name = pipe.draw_kernel_name()   # the kernel csa_draw_async launches (matches rocprofv3 names)
    split = pipe.split_draw and args.pack_on != "fused"   # separate pick-list draw + pack kernels
    W = enc.W
    # distinct-panel exchange buffers (fixed-capacity owner segments: no host sync per step)
    # 24-byte keys (hash + global panel index; hash matches re-drawn on the owner) unless
    # --exchange bitmask
    xchg = Dd.PanelExchange(S, W, world, dev, redraw=(enc.handle, k, args.seed, 0) if args.exchange == "keys"
                            else None) if world > 1 else None

    if args.job_panels:
        return run_job(args, world, rank, dev, torch, dist, A, Dd, enc, k, S, inst_dir, pipe, want_pairs, stream,
                       draw_name)

    overlap = not args.no_overlap
    nb = max(args.bufs, 2) if overlap else 1
    ahead = nb - 1                                  # draws enqueued ahead of the counting
    draw_streams = [torch.cuda.Stream(dev) for _ in range(max(args.draw_streams, 1))] if overlap else [stream]
    pbufs = [pipe.panels] + [torch.empty_like(pipe.panels) for _ in range(nb - 1)]
    hbufs = [pipe.hashes] + [torch.empty_like(pipe.hashes) for _ in range(nb - 1)]
    pack_on_count = split and args.pack_on == "count"
    kbufs = ([pipe.picks] + [torch.empty_like(pipe.picks) for _ in range(nb - 1)]) if pack_on_count else None
    # XT from the draw (the register kernels' fused pack): one XT buffer per panel buffer, since the next
    # draws write theirs while this step's pair kernel reads
    xt_draw = want_pairs and not split and args.xt_from == "draw" and draw_name.startswith(("draw_lane", "draw_solo"))
    xbufs = ([pipe.xt] + [torch.empty_like(pipe.xt) for _ in range(nb - 1)]) if xt_draw else None
    fused_xt = [False] * nb      # did the draw of buffer b write its XT
    drawn = [torch.cuda.Event() for _ in range(nb)]    # draw + pack of the buffer finished (draw stream)
    counted = [torch.cuda.Event() for _ in range(nb)]  # counting of the buffer finished (counting stream)
    stages = ["draw", "pack", "xt_count", "pairs", "unique", "exchange"]
    with torch.cuda.stream(stream):
        pipe.status.zero_()
    last = {"unique": pipe.unique}

    def Ev():
        return torch.cuda.Event(enable_timing=True)

    mode = {"serial": not overlap}

    def enqueue_draw(j, rec):
        b = j % nb
        ds = stream if mode["serial"] else draw_streams[j % len(draw_streams)]
        ds.wait_event(counted[b])                 # step j - nb is done reading this buffer
        pipe.panels, pipe.hashes = pbufs[b], hbufs[b]
        if pack_on_count:
            pipe.picks = kbufs[b]
        begin = (j * world + rank) * S            # global panel indices, distinct per step and rank
        e = [Ev(), Ev(), Ev()] if rec is not None else None
        if e:
            e[0].record(ds)
        if split:
            pipe.draw_picks(args.seed, begin, S, stream=ds)
            if e:
                e[1].record(ds)
            if not pack_on_count:
                pipe.pack(S, stream=ds)
        elif xt_draw:
            pipe.xt = xbufs[b]
            fused_xt[b] = pipe.draw_xt(args.seed, begin, S, stream=ds)
            if e:
                e[1].record(ds)
        else:
            pipe.draw(args.seed, begin, S, stream=ds)
            if e:
                e[1].record(ds)
        if e:
            e[2].record(ds)
            rec[j] = {"draw": (e[0], e[1]), "pack": (e[1], e[2])}
        drawn[b].record(ds)

    def enqueue_count(j, rec):
        b = j % nb
        stream.wait_event(drawn[b])
        pipe.panels, pipe.hashes = pbufs[b], hbufs[b]
        e = [Ev() for _ in range(6)] if rec is not None else None
        pipe.reset(status=False, pairs=False)
        if e:
            e[5].record(stream)
        if pack_on_count:
            pipe.picks = kbufs[b]
            pipe.pack(S, stream=stream)
            if e:
                rec[j]["pack"] = (e[5], e[0])
        if e:
            e[0].record(stream)
        if xt_draw:
            pipe.xt = xbufs[b]
        if not fused_xt[b]:
            pipe.transpose_count(S)
        if e:
            e[1].record(stream)
        if want_pairs:
            # the pair matrix is stored (overwrite), not zero-filled and added; with the draws of the
            # next steps in flight on the other stream the per-CU pair kernel takes its 256-register
            # form, which leaves room for a draw workgroup beside it
            pipe.pair_counts(S, overwrite=True, shared=overlap)
            if fused_xt[b]:
                pipe.counts_from_pairs()     # the step's counts: the stored pair matrix's diagonal
        if e:
            e[2].record(stream)
        if world == 1:
            pipe.unique_count(S)
        if e:
            e[3].record(stream)
        if world > 1:
            with torch.cuda.stream(stream):   # collectives order on the current stream
                last["unique"] = Dd.combine(pipe.counts, pipe.pairs, pipe.hashes[: 2 * S], pipe.panels[: S * W], W,
                                            exchange=xchg, stream=stream, pair_bound=S * world,
                                            status=pipe.status, panel_begin=(j * world + rank) * S)[2]
        if e:
            e[4].record(stream)
            rec[j].update({"xt_count": (e[0], e[1]), "pairs": (e[1], e[2]), "unique": (e[2], e[3]),
                           "exchange": (e[3], e[4])})
        counted[b].record(stream)

    def run_steps(first, count, rec=None):
        """Steps first .. first+count-1: draws `ahead` steps before their counting."""
        for j in range(first, min(first + ahead, first + count)):
            enqueue_draw(j, rec)
        for j in range(first, first + count):
            if j + ahead < first + count and ahead:
                enqueue_draw(j + ahead, rec)
            if not ahead:
                enqueue_draw(j, rec)
            enqueue_count(j, rec)

    run_steps(0, args.warmup)
    torch.cuda.synchronize()
    pipe.check_status()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    A.draw_stats(enc, reset=True)     # SelectionErrors / rejections of the timed draws only
    log = {}
    t0 = time.perf_counter()
    run_steps(args.warmup, args.steps, log)
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
    checks.update({"last_step_" + key: v for key, v in digests(pipe.counts, pipe.pairs if want_pairs else None,
                                                                 enc.n).items()})
    # draw statistics of the timed steps, summed over ranks
    st = torch.tensor(list(A.draw_stats(enc).values()), dtype=torch.int64, device=dev)
    if world > 1:
        Dd._all_reduce(st)
    draw_stats = dict(zip(A.STAT_KEYS, (int(x) for x in st.cpu().tolist())))
    draw_stats["panels"] = S * world * args.steps
    if world > 1:
        # the one-process multi-device path over the same N GPUs (csa_legacy_sample_devices: a replica
        # of the instance per device, peer copies + adds on device 0, exact union of the local distinct
        # sets) for the last timed step's global panel range must equal the rank-sharded result
        dist.barrier()
        if rank == 0:
            j = args.warmup + args.steps - 1
            ndev = max(torch.cuda.device_count(), 1)
            devs = [(dev_index + s_) % ndev for s_ in range(world)]
            try:
                raw = A.legacy_sample_raw(enc, k, S * world, args.seed, panel_begin=j * world * S,
                                          want_pairs=want_pairs, want_panels=False, devices=devs)
                got_c = pipe.counts.cpu().numpy()
                same = bool((raw.counts == got_c).all()) and raw.unique == checks["last_step_unique"]
                if want_pairs:
                    import numpy as np
                    got_p = pipe.pairs.view(enc.n, enc.n).cpu().numpy()
                    same = same and bool(np.array_equal(np.triu(raw.pairs), np.triu(got_p)))
                checks["sample_devices"] = {"devices": devs, "panels": S * world, "unique": raw.unique,
                                            "equal_to_rank_sharded": same}
            except Exception as e:   # a check after the timed region: report it, never strand the other ranks
                checks["sample_devices"] = {"devices": devs, "error": "%s: %s" % (type(e).__name__, e)}
        dist.barrier()

    def stage_times(rec):
        out = {s: 0.0 for s in stages}
        for evs in rec.values():
            for s in stages:
                if s in evs:
                    out[s] += evs[s][0].elapsed_time(evs[s][1]) / len(rec)
        return out

    # stage times inside the timed region (HIP events on the streams the kernels run on); the
    # counting kernels share the CUs with the next steps' draws there.  A short serial pass AFTER
    # the timed region (not part of `value`) measures every kernel alone on the device.
    stage_pipe = stage_times(log)
    # the draw stream's busy fraction in the timed region: ~1 when the host never lets it starve
    # (draws are enqueued `ahead` steps before the counting / exchange that may block the host)
    draw_busy = sum(ev["draw"][0].elapsed_time(ev["draw"][1]) + (ev["pack"][0].elapsed_time(ev["pack"][1])
                                                                  if not pack_on_count else 0.0)
                    for ev in log.values()) / (elapsed * 1e3) if log else None
    iso = {}
    if overlap and args.iso_steps:
        torch.cuda.synchronize()
        ahead_saved, ahead, mode["serial"] = ahead, 0, True     # every kernel alone, one stream
        run_steps(args.warmup + args.steps, args.iso_steps, iso)
        ahead, mode["serial"] = ahead_saved, False
        torch.cuda.synchronize()
        pipe.check_status()
    stage_ms = stage_times(iso) if iso else stage_pipe
    n = enc.n
    npad = pipe.npad
    nblk = (S + 63) // 64
    draw_bytes = S * 2 * k if split else S * (8 * W + 16)   # pick lists written (or bitmasks + hashes)
    if any(fused_xt):
        draw_bytes += ((S + 63) // 64) * pipe.npad * 8    # + the XT operand it writes (fused pack)
    pack_bytes = S * (2 * k + 8 * W + 16)                  # read the pick lists, write panels + hashes
    xt_bytes = S * 8 * W + nblk * npad * 8 + n * 8         # read panels, write transposed bits + counts
    pair_ops = S * n * (n + 1)                             # triangle form of 2*S*n^2
    uniq_bytes = S * (16 + 8 * 2)                          # hashes + index / histogram traffic (approx.)

    def gbs(b, ms):
        return b / (ms * 1e-3) / 1e9 if ms > 0 else 0.0

    kernels = {
        "draw": {"kernel": draw_name, "ms": stage_ms["draw"],
                 "panels_per_s": S / (stage_ms["draw"] * 1e-3) if stage_ms["draw"] else 0,
                 "bound": "issue (VALU/LDS latency)", "hbm_GBps": gbs(draw_bytes, stage_ms["draw"]),
                 "algorithmic_bytes": draw_bytes},
        "xt_count": {"kernel": "xt_count_kernel", "ms": stage_ms["xt_count"], "hbm_GBps": gbs(xt_bytes, stage_ms["xt_count"]),
                     "frac": gbs(xt_bytes, stage_ms["xt_count"]) * 1e9 / HBM_PEAK},
        "unique": {"ms": stage_ms["unique"], "hbm_GBps": gbs(uniq_bytes, stage_ms["unique"])},
    }
    if split:
        kernels["pack"] = {"kernel": "picks_pack_kernel", "ms": stage_ms["pack"],
                           "hbm_GBps": gbs(pack_bytes, stage_ms["pack"]),
                           "frac": gbs(pack_bytes, stage_ms["pack"]) * 1e9 / HBM_PEAK}
    if want_pairs:
        tops = pair_ops / (stage_ms["pairs"] * 1e-3) / 1e12 if stage_ms["pairs"] else 0.0
        kernels["pairs_mfma"] = {"ms": stage_ms["pairs"], "engine": args.pair_engine, "operands": engine_desc,
                                 "TOPs": tops, "ops_per_launch": pair_ops,
                                 "mfma_util": tops * 1e12 / engine_peak, "peak_TOPs": engine_peak / 1e12,
                                 "int8_peak_equiv": tops * 1e12 / I8_MFMA_PEAK,
                                 "note": "ops = S*n*(n+1) (upper triangle incl. diagonal of 2*S*n^2); "
                                         "ms includes the partial-block reduce kernel"}
    if world > 1:
        kernels["exchange"] = {"ms": stage_ms["exchange"], "form": args.exchange,
                               "bytes_sent_per_rank": xchg.bytes_sent()}
    for key, st in (("draw", "draw"), ("pack", "pack"), ("xt_count", "xt_count"), ("unique", "unique"),
                    ("pairs_mfma", "pairs"), ("exchange", "exchange")):
        if key in kernels:
            kernels[key]["ms_in_timed_region"] = stage_pipe[st]
    kernel_timing = ("'ms' = each kernel alone (serial pass of %d steps after the timed region); "
                     "'ms_in_timed_region' = HIP events on the launch streams inside the timed region, "
                     "where the counting kernels share the CUs with the next steps' draws" % len(iso)
                     ) if iso else "HIP events on the launch stream inside the timed region (serial steps)"
    dominant = max(("draw", "pack", "xt_count", "pairs", "unique"), key=lambda s: stage_pipe[s])
    pmc = load_pmc(args.config)
    sha = source_sha()
    pmc_ok = bool(pmc and pmc.get("source_sha") == sha and pmc.get("panels") == S)
    # the roofline's kernel duration is the one inside the timed region (what rocprofv3 averages)
    if dominant == "pairs":
        ach = pair_ops / (stage_pipe["pairs"] * 1e-3) / 1e12
        roof = {"kernel": "pair_mfma_kernel", "bound": "mfma", "achieved": ach, "peak": engine_peak / 1e12,
                "unit": "TFLOP/s", "frac": ach * 1e12 / engine_peak, "traffic": None}
    else:
        name = {"draw": draw_name, "pack": "picks_pack_kernel", "xt_count": "xt_count_kernel",
                "unique": "uq_dedupe_kernel"}[dominant]
        b = {"draw": draw_bytes, "pack": pack_bytes, "xt_count": xt_bytes, "unique": uniq_bytes}[dominant]
        ach = gbs(b, stage_pipe[dominant])
        traffic = None
        pk = (pmc or {}).get("per_kernel", {}).get(name)
        if pk and pmc_ok:
            traffic = pk.get("hbm_bytes_per_launch")     # rocprofv3 --pmc FETCH/WRITE passes of these kernels
        roof = {"kernel": name, "bound": "hbm", "achieved": ach, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                "frac": ach * 1e9 / HBM_PEAK, "traffic": traffic, "algorithmic_bytes": b}
        if dominant == "draw":
            roof["note"] = ("the draw kernel has no HBM or MFMA roof: it is bound by VALU issue; 'achieved' is its "
                            "algorithmic output bytes (%s) over its in-region time (the HBM "
                            "framing the contract asks for); roofline.valu is the binding roof: its VALU "
                            "wave-instructions per second (rocprofv3 SQ_INSTS_VALU of these sources) over the "
                            "rate the kernel's class mix allows (tools/valu_budget.py: single-issue VALU 4.3, "
                            "dual-issue 2.47 SIMD cycles per wave-instruction, tools/coissue.hip); issue_frac_2cyc "
                            "is the same count priced at 2 cycles per wave-instruction") % ("2k B of pick list per panel" if split else
                                             "8W + 16 B of packed panel and hash%s per panel" % (
                                                 " + n_pad / 8 B of the XT operand it writes" if any(fused_xt) else ""))
            if pmc_ok and pmc.get("draw_issue") and pmc.get("draw_kernel") == draw_name:
                kernels["draw"]["pmc_issue"] = pmc["draw_issue"]
                roof["issue_frac_2cyc"] = pmc["draw_issue"].get("valu_issue_frac")
                roof["mean_waves_per_simd"] = pmc["draw_issue"].get("mean_waves_per_simd")
                # the roof that binds: VALU instructions of this kernel (PMC, same sources) per second in
                # the timed region vs the rate its class mix allows at the clock it runs at (every
                # single-issue instruction 4.3 cycles of its SIMD, every dual-issue one 2.47 cycles);
                # single_issue: one VALU per 4 cycles per SIMD (the quad rate, SQ_ACTIVE_INST_VALU)
                vb = load_valu_budget(args.config)
                if vb and stage_pipe["draw"] > 0:
                    vpp = pmc["draw_issue"]["valu_insts_per_panel"]
                    clk = pmc["draw_issue"]["clock_GHz"] * 1e9
                    rate = vpp * S / (stage_pipe["draw"] * 1e-3)
                    peak = vpp / vb["budget_class_weighted_cycles_per_panel"] * 1024 * clk
                    roof["valu"] = {"bound": "valu_issue", "achieved": rate, "peak": peak,
                                    "unit": "wave-instructions/s", "frac": rate / peak,
                                    "single_issue_peak": 1024 * clk / 4, "single_issue_frac": rate / (1024 * clk / 4),
                                    "valu_insts_per_panel": vpp, "half_rate_frac": vb["valu_per_panel"]["half_frac"],
                                    "clock_GHz": clk / 1e9,
                                    "pmc_valu_active_frac": pmc["draw_issue"].get("valu_active_frac"),
                                    "peak_source": "profiles/valu_budget_%s.json (tools/valu_budget.py: class-weighted "
                                                   "budget of the kernel's dynamic VALU mix)" % args.config}
    roof["pmc_source_sha"] = sha
    roof["pmc_matches_sources"] = pmc_ok

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
            "pipeline": ("draws on their own stream, %d steps ahead of the counting%s" % (
                ahead, " and the exchange" if world > 1 else "")) if overlap else "serial",
            "xt_operand": ("written by the draw kernel's fused pack (one XT buffer per panel buffer); counts = "
                           "the stored pair matrix's diagonal") if any(fused_xt) else "xt_count_kernel"},
        "roofline": roof,
        "kernels": kernels,
        "kernel_timing": kernel_timing,
        "checks": checks,
        "draw_stats": draw_stats,
        "draw_stream_busy": draw_busy,
    }
    if want_pairs:
        result["xtx_mfma_util"] = kernels["pairs_mfma"]["mfma_util"]
        result["xtx_int8_peak_equiv"] = kernels["pairs_mfma"]["int8_peak_equiv"]
    if rank == 0 and world == 1 and not args.no_api and args.config == "sf_e_110":
        result["api"] = api_leg(P, A, inst, 10 ** 6, args.seed)
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
