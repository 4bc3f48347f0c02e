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
  * distinct panels    every 128-bit panel hash goes to its OWNER rank
                       (h1 % world) with one all_to_all (buckets from
                       csa_hash_buckets_async); the owner counts its distinct
                       hashes with the device hash table (csa_unique_hashes_async),
                       then all_reduce(SUM).  Exact within a rank (bitmask compare in
                       the single-rank path); across ranks two panels merge when
                       their 128-bit hashes agree (collision odds ~S^2/2^129).
On CPU (gloo, tests) the same exchange runs on host tensors and the owner
dedupe uses numpy; ``panel_hashes`` mirrors the device hash for that path.
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
    """Host mirror of the draw kernel's 128-bit panel hash: uint64[S, 2] from uint64[S, W]."""
    p = np.ascontiguousarray(panels, np.uint64)
    S, W = p.shape
    w = np.arange(W, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h1 = _fmix_a(p ^ (w * np.uint64(0x9E3779B97F4A7C15))).sum(axis=1, dtype=np.uint64)
        h2 = _fmix_b(p + (w + np.uint64(1)) * np.uint64(0xD6E8FEB86659FD93)).sum(axis=1, dtype=np.uint64)
    return np.stack([h1, h2], axis=1)


def dedupe_hash_partition(all_hashes, world, r):
    """Number of distinct 128-bit hashes owned by rank r (owner = h1 mod world)."""
    h = np.asarray(all_hashes, np.uint64).reshape(-1, 2)
    mine = h[(h[:, 0] % np.uint64(world)) == np.uint64(r)]
    if len(mine) == 0:
        return 0
    return int(len(np.unique(mine, axis=0)))


class HashTable:
    """Reusable device table for csa_unique_hashes_async (grows on demand)."""

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
    """gloo has no all_to_all for device tensors: rehearsals (CSA_BENCH_BACKEND=gloo) go via host."""
    import torch.distributed as dist
    return t.is_cuda and dist.get_backend() != "nccl"


def exchange_hashes(hashes, stream=None):
    """Send every 128-bit panel hash to its owner rank (h1 % world) with one all_to_all.

    hashes: int64[2*S_local] on the device (buckets from csa_hash_buckets_async) or on the host
    (numpy bucketing, gloo tests).  Returns int64[2*S_owned], the hashes this rank owns."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    n = hashes.numel() // 2
    if hashes.is_cuda:
        from . import _native as N
        out = torch.empty_like(hashes)
        counts = torch.empty(world, dtype=torch.int64, device=hashes.device)
        cursor = torch.empty(world, dtype=torch.int64, device=hashes.device)
        sp = ctypes.c_void_p((stream or torch.cuda.current_stream(hashes.device)).cuda_stream)
        N.check(N.lib().csa_hash_buckets_async(N.ptr(hashes), n, world, N.ptr(out), N.ptr(counts), N.ptr(cursor), sp))
    else:
        h = hashes.numpy().view(np.uint64).reshape(-1, 2)
        owner = (h[:, 0] % np.uint64(world)).astype(np.int64)
        order = np.argsort(owner, kind="stable")
        out = torch.from_numpy(np.ascontiguousarray(h[order]).view(np.int64).reshape(-1))
        counts = torch.from_numpy(np.bincount(owner, minlength=world).astype(np.int64))
    via_host = _host_collectives(out)
    send_counts = counts.cpu() if via_host else counts
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts)
    in_splits = [2 * int(c) for c in send_counts.tolist()]
    out_splits = [2 * int(c) for c in recv_counts.tolist()]
    src = out.cpu() if via_host else out
    recv = torch.empty(sum(out_splits), dtype=torch.int64, device=src.device)
    dist.all_to_all_single(recv, src, out_splits, in_splits)
    return recv.to(hashes.device) if via_host else recv


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


def combine(counts, pairs, hashes, table=None, stream=None, pair_bound=None):
    """Exchange steps for this rank; returns (counts, pairs, unique_tensor).

    counts int64[n], pairs int64[n*n] or None, hashes int64[2*S_local] (this rank's
    panel hashes).  Counts and pairs: all_reduce(SUM).  Distinct panels: every hash goes to
    its owner rank (exchange_hashes, one all_to_all), the owner counts its distinct hashes
    (device hash table on GPU tensors, numpy on CPU), all_reduce(SUM) of the counts.
    """
    import torch
    import torch.distributed as dist
    if _host_collectives(counts):
        h = counts.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM)
        counts.copy_(h)
    else:
        dist.all_reduce(counts, op=dist.ReduceOp.SUM)
    if pairs is not None:
        _all_reduce_pairs(pairs, pair_bound, stream)
    mine = exchange_hashes(hashes, stream)
    if mine.is_cuda:
        from . import _native as N
        if table is None:
            table = HashTable(mine.numel() // 2, mine.device)
        table.ensure(mine.numel() // 2)
        table.count.zero_()
        sp = ctypes.c_void_p((stream or torch.cuda.current_stream(mine.device)).cuda_stream)
        N.check(N.lib().csa_unique_hashes_async(N.ptr(mine), mine.numel() // 2, 1, 0, N.ptr(table.table),
                                                table.slots, N.ptr(table.count), sp))
        u = table.count.clone()
    else:
        m = mine.numpy().view(np.uint64).reshape(-1, 2)
        u = torch.tensor([int(len(np.unique(m, axis=0))) if len(m) else 0], dtype=torch.int64)
    if _host_collectives(u):
        h = u.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM)
        u.copy_(h)
    else:
        dist.all_reduce(u, op=dist.ReduceOp.SUM)
    return counts, pairs, u


def legacy_probabilities_distributed(instance, iterations, random_seed, keep_panels=False):
    """analysis.py:162-191 with the panels sharded over the ranks of the default group."""
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
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", r)))
    pipe = DevicePipeline(enc, instance.k, max(local, 1), want_pairs=True, want_unique=True)
    pipe.reset()
    if local:
        pipe.run(random_seed, begin, local)
    pipe.check_status()
    counts, pairs, u = combine(pipe.counts, pipe.pairs, pipe.hashes[: 2 * local], pair_bound=S)
    raw = A.LegacyRaw(counts.cpu().numpy(), pairs.cpu().numpy().reshape(enc.n, enc.n), int(u.item()), None, None)
    return A.finish(instance, enc, raw, S)
