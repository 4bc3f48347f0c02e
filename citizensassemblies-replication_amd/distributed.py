"""Multi-GPU LEGACY estimation: one process per GPU, torch.distributed over RCCL.

Sharding (DESIGN.md "Multi-GPU"): the global panel range [0, S) is cut into
contiguous per-rank ranges.  Every random draw is keyed by the GLOBAL panel
index (Philox counter = (step, attempt, panel)), so the union of the shards is
bit-identical to a single-GPU run for any world size; no data-path collective
is needed for the draw itself.

Exchange steps (the only collectives on the path):
  * per-person counts  all_reduce(SUM) int64[n]
  * pair counts        all_reduce(SUM) of the upper triangle packed to int32
                       (csa_pairs_pack/unpack_async; int64[n*n] if a count may
                       reach 2^31)
  * distinct panels    every panel -- its 128-bit hash AND its W-word bitmask --
                       goes to its OWNER rank (h1 % world; equal panels have
                       equal hashes, so all copies of a panel meet at one owner)
                       with all_to_all (buckets from csa_hash_buckets_async); the
                       owner counts its distinct panels with csa_unique_async,
                       which compares bitmasks on a hash match, so the count is
                       exact (analysis.py:171,186: a set of sorted tuples); then
                       all_reduce(SUM) of the owners' counts.
The bucket sizes are negotiated with a small all_to_all whose result the host
reads (the only host synchronisation of the exchange); bench.py enqueues the
next steps' draws before it, so the draw stream never waits for it.
On CPU (gloo, tests) the same exchange runs on host tensors: numpy bucketing by
owner and an exact numpy dedupe of the bitmasks; ``panel_hashes`` mirrors the
device hash for that path.
"""
import ctypes
import os

import numpy as np

M64 = 0xFFFFFFFFFFFFFFFF


def world_size():
    try:
        import torch.distributed as dist
    except Exception:
        return 1
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size()
    return 1


def rank():
    import torch.distributed as dist
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def shard_range(S, world, r):
    """Contiguous shard [begin, end) of S panels for rank r of world."""
    per, extra = divmod(int(S), int(world))
    begin = r * per + min(r, extra)
    return begin, begin + per + (1 if r < extra else 0)


def _fmix_a(z):
    z = z ^ (z >> np.uint64(30))
    z = z * np.uint64(0xBF58476D1CE4E5B9)
    z = z ^ (z >> np.uint64(27))
    z = z * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def _fmix_b(z):
    z = z ^ (z >> np.uint64(33))
    z = z * np.uint64(0xFF51AFD7ED558CCD)
    z = z ^ (z >> np.uint64(33))
    z = z * np.uint64(0xC4CEB9FE1A85EC53)
    return z ^ (z >> np.uint64(33))


def panel_hashes(panels):
    """Host mirror of the device 128-bit panel hash: uint64[S, 2] from uint64[S, W]."""
    p = np.ascontiguousarray(panels, np.uint64)
    S, W = p.shape
    w = np.arange(W, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h1 = _fmix_a(p ^ (w * np.uint64(0x9E3779B97F4A7C15))).sum(axis=1, dtype=np.uint64)
        h2 = _fmix_b(p + (w + np.uint64(1)) * np.uint64(0xD6E8FEB86659FD93)).sum(axis=1, dtype=np.uint64)
    return np.stack([h1, h2], axis=1)


def owner_buckets(hashes, panels, world):
    """Host mirror of csa_hash_buckets_async: (hashes, panels, counts) in owner-major order,
    owner = h1 % world."""
    h = np.asarray(hashes, np.uint64).reshape(-1, 2)
    p = np.asarray(panels, np.uint64).reshape(len(h), -1)
    owner = (h[:, 0] % np.uint64(world)).astype(np.int64)
    order = np.argsort(owner, kind="stable")
    return h[order], p[order], np.bincount(owner, minlength=world).astype(np.int64)


def distinct_exact(hashes, panels):
    """Host mirror of csa_unique_async: distinct panels, equal iff hash AND bitmask are equal."""
    p = np.asarray(panels, np.uint64)
    if len(p) == 0:
        return 0
    h = np.asarray(hashes, np.uint64).reshape(len(p), 2)
    return int(len(np.unique(np.concatenate([h, p.reshape(len(p), -1)], axis=1), axis=0)))


class HashTable:
    """Reusable device table + count for csa_unique_async (grows on demand)."""

    def __init__(self, max_hashes, device):
        import torch
        self.device = device
        self.count = torch.zeros(1, dtype=torch.int64, device=device)
        self.slots = 0
        self.ensure(max_hashes)

    def ensure(self, n_hashes):
        import torch
        slots = 64
        while slots < 2 * max(int(n_hashes), 1):
            slots <<= 1
        if slots > self.slots:
            self.slots = slots
            self.table = torch.empty(slots, dtype=torch.int64, device=self.device)


def _host_collectives(t):
    """gloo rehearsals of the device path (CSA_BENCH_BACKEND=gloo) run the collectives on host copies."""
    import torch.distributed as dist
    return t.is_cuda and dist.get_backend() != "nccl"


def exchange_panels(hashes, panels, W, stream=None):
    """Send every panel (128-bit hash + W-word bitmask) to its owner rank h1 % world.

    hashes: int64[2*S_local], panels: int64[S_local*W], both on the device (buckets from
    csa_hash_buckets_async) or on the host (numpy bucketing).  Returns (hashes, panels) this rank
    owns: int64[2*m], int64[m*W]."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    n = hashes.numel() // 2
    if hashes.is_cuda:
        from . import _native as N
        out_h = torch.empty_like(hashes)
        out_p = torch.empty(max(n * W, 1), dtype=torch.int64, device=hashes.device)
        counts = torch.empty(world, dtype=torch.int64, device=hashes.device)
        cursor = torch.empty(world, dtype=torch.int64, device=hashes.device)
        sp = ctypes.c_void_p((stream or torch.cuda.current_stream(hashes.device)).cuda_stream)
        N.check(N.lib().csa_hash_buckets_async(N.ptr(hashes), N.ptr(panels), n, W, world, N.ptr(out_h),
                                               N.ptr(out_p), N.ptr(counts), N.ptr(cursor), sp))
        out_p = out_p[: n * W]
    else:
        h, p, c = owner_buckets(hashes.numpy().view(np.uint64), panels.numpy().view(np.uint64).reshape(n, W), world)
        out_h = torch.from_numpy(np.ascontiguousarray(h).view(np.int64).reshape(-1))
        out_p = torch.from_numpy(np.ascontiguousarray(p).view(np.int64).reshape(-1))
        counts = torch.from_numpy(c)
    via_host = _host_collectives(out_h)
    send_counts = counts.cpu() if via_host else counts
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts)
    sc, rc = send_counts.tolist(), recv_counts.tolist()   # the exchange's one host synchronisation
    src_h = out_h.cpu() if via_host else out_h
    src_p = out_p.cpu() if via_host else out_p
    recv_h = torch.empty(2 * sum(rc), dtype=torch.int64, device=src_h.device)
    recv_p = torch.empty(W * sum(rc), dtype=torch.int64, device=src_p.device)
    dist.all_to_all_single(recv_h, src_h, [2 * c for c in rc], [2 * c for c in sc])
    dist.all_to_all_single(recv_p, src_p, [W * c for c in rc], [W * c for c in sc])
    if via_host:
        return recv_h.to(hashes.device), recv_p.to(hashes.device)
    return recv_h, recv_p


def _all_reduce_pairs(pairs, pair_bound, stream):
    """all_reduce(SUM) of the pair counts.  On GPU tensors with every summed count < 2^31
    (``pair_bound``: the panels of the whole job) only the upper triangle travels, as int32."""
    import torch
    import torch.distributed as dist
    n = int(round(pairs.numel() ** 0.5))
    if pairs.is_cuda and pair_bound is not None and pair_bound < 2 ** 31 and not _host_collectives(pairs):
        from . import _native as N
        sp = ctypes.c_void_p((stream or torch.cuda.current_stream(pairs.device)).cuda_stream)
        packed = torch.empty(n * (n + 1) // 2, dtype=torch.int32, device=pairs.device)
        N.check(N.lib().csa_pairs_pack_async(N.ptr(pairs), n, N.ptr(packed), sp))
        dist.all_reduce(packed, op=dist.ReduceOp.SUM)
        N.check(N.lib().csa_pairs_unpack_async(N.ptr(packed), n, N.ptr(pairs), sp))
    elif _host_collectives(pairs):
        h = pairs.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM)
        pairs.copy_(h)
    else:
        dist.all_reduce(pairs, op=dist.ReduceOp.SUM)


def _all_reduce(t):
    import torch.distributed as dist
    if _host_collectives(t):
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)


def combine(counts, pairs, hashes, panels, W, table=None, stream=None, pair_bound=None, status=None):
    """Exchange steps for this rank; returns (counts, pairs, unique_tensor).

    counts int64[n], pairs int64[n*n] or None, hashes int64[2*S_local] and panels
    int64[S_local*W] (this rank's panels).  Counts and pairs: all_reduce(SUM).  Distinct
    panels: every panel goes to its owner rank (exchange_panels), the owner counts its distinct
    panels exactly (device: csa_unique_async with bitmask comparison, table overflow reported in
    ``status``; host: numpy), all_reduce(SUM) of the counts.
    """
    import torch
    _all_reduce(counts)
    if pairs is not None:
        _all_reduce_pairs(pairs, pair_bound, stream)
    mine_h, mine_p = exchange_panels(hashes, panels, W, stream)
    m = mine_h.numel() // 2
    if mine_h.is_cuda:
        from . import _native as N
        if table is None:
            table = HashTable(m, mine_h.device)
        table.ensure(m)
        table.count.zero_()
        sp = ctypes.c_void_p((stream or torch.cuda.current_stream(mine_h.device)).cuda_stream)
        N.check(N.lib().csa_unique_async(N.ptr(mine_h), N.ptr(mine_p), m, W, N.ptr(table.table), table.slots,
                                         N.ptr(table.count), N.ptr(status), sp))
        u = table.count.clone()
    else:
        u = torch.tensor([distinct_exact(mine_h.numpy().view(np.uint64), mine_p.numpy().view(np.uint64).reshape(m, W))],
                         dtype=torch.int64)
    _all_reduce(u)
    return counts, pairs, u


def gather_panels(panels, S, W):
    """All ranks' shards (contiguous global ranges, shard_range) -> uint64[S, W] on every rank."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    per = shard_range(S, world, 0)[1]
    buf = torch.zeros(per * W, dtype=torch.int64, device=panels.device)
    buf[: panels.numel()] = panels
    src = buf.cpu() if _host_collectives(buf) else buf
    parts = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(parts, src)
    rows = []
    for r, t in enumerate(parts):
        b, e = shard_range(S, world, r)
        rows.append(t.cpu().numpy().view(np.uint64).reshape(per, W)[: e - b])
    return np.concatenate(rows) if rows else np.zeros((0, W), np.uint64)


def legacy_probabilities_distributed(instance, iterations, random_seed, keep_panels=True):
    """analysis.py:162-191 with the panels sharded over the ranks of the default group.  Every rank
    returns the whole job's results; with ``keep_panels`` every rank gathers all panels so that
    ``found_panels`` iterates like the reference's set (costs S*W*8 bytes per rank)."""
    import torch
    from . import analysis as A
    from .device import DevicePipeline
    from .instance import encode
    world, r = world_size(), rank()
    S = int(iterations)
    A.seed(random_seed)
    A.STREAM.take_panels(S)
    enc = encode(instance.categories, instance.agents)
    enc.check_quotas(instance.k)
    begin, end = shard_range(S, world, r)
    local = end - begin
    # one process per GPU (LOCAL_RANK); the modulo lets rehearsals put several ranks on one device
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", r)) % max(torch.cuda.device_count(), 1))
    pipe = DevicePipeline(enc, instance.k, max(local, 1), want_pairs=True, want_unique=True)
    pipe.reset()
    if local:
        pipe.draw(random_seed, begin, local)
        pipe.transpose_count(local)
        pipe.pair_counts(local)
    pipe.check_status()
    counts, pairs, u = combine(pipe.counts, pipe.pairs, pipe.hashes[: 2 * local], pipe.panels[: local * enc.W],
                               enc.W, pair_bound=S, status=pipe.status)
    pipe.check_status()
    panels = gather_panels(pipe.panels[: local * enc.W], S, enc.W) if keep_panels else None
    raw = A.LegacyRaw(counts.cpu().numpy(), pairs.cpu().numpy().reshape(enc.n, enc.n), int(u.item()), panels, None)
    return A.finish(instance, enc, raw, S)
