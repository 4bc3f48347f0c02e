"""Multi-GPU LEGACY estimation: one process per GPU, torch.distributed over RCCL.

Sharding (DESIGN.md "Multi-GPU"): the global panel range [0, S) is cut into
contiguous per-rank ranges.  Every random draw is keyed by the GLOBAL panel
index (Philox counter = (step, attempt, panel)), so the union of the shards is
bit-identical to a single-GPU run for any world size; no data-path collective
is needed for the draw itself.

Exchange steps (the only collectives on the path):
  * per-person counts  all_reduce(SUM) int64[n]
  * pair counts        all_reduce(SUM) int64[n*n]   (upper triangle meaningful)
  * distinct panels    all_gather of every rank's 128-bit panel hashes; rank r
                       counts the distinct hashes it OWNS (h1 % world == r) with
                       the device hash table (csa_unique_hashes_async), then
                       all_reduce(SUM).  Exact within a rank (bitmask compare in
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


def _gather_hashes(hashes):
    """all_gather of variable-length int64 hash tensors -> one concatenated tensor."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    n_local = torch.tensor([hashes.numel()], dtype=torch.int64, device=hashes.device)
    sizes = [torch.zeros_like(n_local) for _ in range(world)]
    dist.all_gather(sizes, n_local)
    sizes = [int(s.item()) for s in sizes]
    maxn = max(sizes) if sizes else 0
    padded = torch.zeros(max(maxn, 1), dtype=torch.int64, device=hashes.device)
    padded[: hashes.numel()] = hashes
    gathered = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(gathered, padded)
    return torch.cat([g[:s] for g, s in zip(gathered, sizes)])


class HashTable:
    """Reusable device table for csa_unique_hashes_async."""

    def __init__(self, max_hashes, device):
        import torch
        slots = 64
        while slots < 2 * max(int(max_hashes), 1):
            slots <<= 1
        self.slots = slots
        self.table = torch.empty(slots, dtype=torch.int64, device=device)
        self.count = torch.zeros(1, dtype=torch.int64, device=device)


def combine(counts, pairs, hashes, table=None, stream=None):
    """Exchange steps for this rank; returns (counts, pairs, unique_tensor).

    counts int64[n], pairs int64[n*n] or None, hashes int64[2*S_local] (this rank's
    panel hashes).  On GPU tensors the owner dedupe runs on the device (``table``
    = HashTable); on CPU tensors (gloo) it runs in numpy.
    """
    import torch
    import torch.distributed as dist
    world, r = dist.get_world_size(), dist.get_rank()
    dist.all_reduce(counts, op=dist.ReduceOp.SUM)
    if pairs is not None:
        dist.all_reduce(pairs, op=dist.ReduceOp.SUM)
    all_h = _gather_hashes(hashes)
    if all_h.is_cuda:
        from . import _native as N
        if table is None:
            table = HashTable(all_h.numel() // 2, all_h.device)
        table.count.zero_()
        sp = ctypes.c_void_p(stream.cuda_stream) if stream is not None else \
            ctypes.c_void_p(torch.cuda.current_stream(all_h.device).cuda_stream)
        N.check(N.lib().csa_unique_hashes_async(N.ptr(all_h), all_h.numel() // 2, world, r, N.ptr(table.table),
                                                table.slots, N.ptr(table.count), sp))
        u = table.count
    else:
        u = torch.tensor([dedupe_hash_partition(all_h.numpy().view(np.uint64), world, r)], dtype=torch.int64)
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
    counts, pairs, u = combine(pipe.counts, pipe.pairs, pipe.hashes[: 2 * local])
    raw = A.LegacyRaw(counts.cpu().numpy(), pairs.cpu().numpy().reshape(enc.n, enc.n), int(u.item()), None, None)
    return A.finish(instance, enc, raw, S)
