"""Multi-GPU LEGACY estimation: one process per GPU, torch.distributed over RCCL.

Sharding (DESIGN.md "Multi-GPU"): the global panel range [0, S) is cut into
contiguous per-rank ranges.  Every random draw is keyed by the GLOBAL panel
index (Philox counter = (step, attempt, panel)), so the union of the shards is
bit-identical to a single-GPU run for any world size; no data-path collective
is needed for the draw itself.

Exchange steps (the only collectives on the path), all
stream-ordered -- the host never waits for the device:
  * per-person counts  all_reduce(SUM) int64[n]
  * pair counts        all_reduce(SUM) of the upper triangle packed to int32
                       (csa_pairs_pack/unpack_async; int64[n*n] if a count may
                       reach 2^31)
  * distinct panels    each rank first reduces its panels to its exact LOCAL
                       distinct set (hash AND bitmask), then sends every one --
                       its 128-bit hash and W-word bitmask -- to its OWNER rank
                       (h1 % world; equal panels have equal hashes, so all copies
                       of a panel meet at one owner).  The segments per owner have
                       a FIXED capacity (binomial bound on a uniform hash, see
                       exchange_capacity), so the three all_to_alls (segment
                       counts, hashes, bitmasks) have equal splits and need no
                       host-side size negotiation (csa_exchange_pack_async).  The
                       owner counts the distinct panels among the valid entries
                       exactly (csa_unique_segments_async: bitmask comparison on a
                       hash match; analysis.py:171,186 is a set of sorted tuples),
                       then all_reduce(SUM).  A segment past its capacity is an
                       error in the status block, never a wrong count.
On CPU (gloo, tests) the same exchange runs on host tensors with numpy mirrors
of the two kernels; ``panel_hashes`` mirrors the device hash for that path.
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


def exchange_capacity(n_local, world):
    """Entries per owner segment for a rank with n_local panels: the distinct panels reaching one
    owner are Binomial(m <= n_local, 1/world) under a uniform hash, so mean + 8 sd + 64 never
    overflows in practice (P < 1e-15 per segment); never more than n_local."""
    n_local, world = max(int(n_local), 1), int(world)
    mean = -(-n_local // world)
    return min(n_local, mean + 8 * int(mean ** 0.5 + 1) + 64)


def local_distinct(hashes, panels):
    """Host mirror of the first stage of csa_exchange_pack_async: the exact distinct rows (hash AND
    bitmask) of uint64[m, 2] / uint64[m, W]."""
    h = np.asarray(hashes, np.uint64).reshape(-1, 2)
    p = np.asarray(panels, np.uint64)
    assert p.ndim == 2 and len(p) == len(h)
    if len(h) == 0:
        return h, p
    u = np.unique(np.concatenate([h, p], axis=1), axis=0)
    return np.ascontiguousarray(u[:, :2]), np.ascontiguousarray(u[:, 2:])


def segment_buckets(hashes, panels, world, cap):
    """Host mirror of csa_exchange_pack_async (panels uint64[m, W]): the local distinct panels in
    fixed-capacity owner segments.  Returns (uint64[world, cap, 2], uint64[world, cap, W], int64[world] counts)."""
    h, p = local_distinct(hashes, panels)
    W = p.shape[1]
    sh = np.zeros((world, cap, 2), np.uint64)
    sp = np.zeros((world, cap, W), np.uint64)
    sc = np.zeros(world, np.int64)
    owner = (h[:, 0] % np.uint64(world)).astype(np.int64) if len(h) else np.zeros(0, np.int64)
    for w in range(world):
        sel = np.nonzero(owner == w)[0]
        if len(sel) > cap:
            raise RuntimeError("distinct-panel exchange: %d panels for owner %d exceed the segment capacity %d"
                               % (len(sel), w, cap))
        sh[w, : len(sel)] = h[sel]
        sp[w, : len(sel)] = p[sel]
        sc[w] = len(sel)
    return sh, sp, sc


def distinct_exact(hashes, panels):
    """Host mirror of csa_unique_async: distinct panels, equal iff hash AND bitmask are equal."""
    p = np.asarray(panels, np.uint64)
    if len(p) == 0:
        return 0
    h = np.asarray(hashes, np.uint64).reshape(len(p), 2)
    return int(len(np.unique(np.concatenate([h, p.reshape(len(p), -1)], axis=1), axis=0)))


def distinct_segments(hashes, panels, counts):
    """Host mirror of csa_unique_segments_async: distinct panels among the valid leading entries of
    each segment (uint64[world, cap, 2], uint64[world, cap, W], counts[world])."""
    h = np.asarray(hashes, np.uint64)
    p = np.asarray(panels, np.uint64)
    c = [int(x) for x in counts]
    hv = np.concatenate([h[w, : c[w]] for w in range(len(c))]) if c else np.zeros((0, 2), np.uint64)
    pv = np.concatenate([p[w, : c[w]] for w in range(len(c))]) if c else np.zeros((0, p.shape[-1]), np.uint64)
    return distinct_exact(hv, pv)


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


def _all_to_all(out, inp):
    """Equal-split all_to_all_single, through host copies for a gloo rehearsal on device tensors."""
    import torch.distributed as dist
    if _host_collectives(inp):
        o = out.cpu()
        dist.all_to_all_single(o, inp.cpu())
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp)


class PanelExchange:
    """The distinct-panel exchange of one rank, buffers sized once for n_local panels of W words.

    ``run(hashes, panels, n, status, stream, panel_begin)`` returns this rank's owner count (a
    1-element int64 tensor, device or host like the inputs); the caller all_reduces it.  Device
    inputs: no host synchronisation, so a caller can enqueue the next steps behind it.

    With ``redraw = (instance handle, k, seed, max_attempts)`` (the draw that made the panels, Philox
    mode) the 24-byte exchange runs: keys (h1, h2, global panel index) instead of bitmasks
    (csa_exchange_keys_async -> two equal-split all_to_alls -> csa_unique_keys_async, which re-draws
    only the hash-matched entries to compare their bitmasks).  Without it, the bitmasks travel
    (csa_exchange_pack_async -> three all_to_alls -> csa_unique_segments_async); host tensors always
    take that form through its numpy mirrors."""

    def __init__(self, n_local, W, world, device, redraw=None):
        import torch
        from . import _native as N
        self.W, self.world, self.device = int(W), int(world), device
        self.n_local = max(int(n_local), 1)
        self.cap = exchange_capacity(self.n_local, self.world)
        self.cuda = torch.device(device).type == "cuda"
        self.redraw = redraw if self.cuda else None
        if not self.cuda:
            return
        i64 = torch.int64
        seg = self.world * self.cap
        sb = int(N.lib().csa_exchange_scratch_bytes(self.n_local))
        self.scratch = torch.empty((sb + 7) // 8, dtype=i64, device=device)
        self.send_c = torch.zeros(self.world, dtype=i64, device=device)
        self.recv_c = torch.zeros_like(self.send_c)
        self.unique = torch.zeros(1, dtype=i64, device=device)
        if self.redraw is not None:
            self.send_k = torch.empty(3 * seg, dtype=i64, device=device)
            self.recv_k = torch.empty_like(self.send_k)
            ob = int(N.lib().csa_unique_keys_scratch_bytes(seg, self.W))
            self.owner_scratch = torch.empty((ob + 7) // 8, dtype=i64, device=device)
            return
        self.send_h = torch.empty(2 * seg, dtype=i64, device=device)
        self.send_p = torch.empty(seg * self.W, dtype=i64, device=device)
        self.recv_h = torch.empty_like(self.send_h)
        self.recv_p = torch.empty_like(self.send_p)
        self.table = HashTable(seg, device)

    def bytes_sent(self):
        """Bytes this rank puts into the all_to_alls per run (segments of every owner, itself included)."""
        per = 24 if self.redraw is not None else 16 + 8 * self.W
        return self.world * self.cap * per + 8 * self.world

    def run(self, hashes, panels, n, status=None, stream=None, panel_begin=0, redraw=None):
        """``redraw`` overrides the constructor's (instance, k, seed, max_attempts) for this run (a
        cached exchange serves calls with different seeds); the form -- keys or bitmasks -- is the
        constructor's."""
        import torch
        n = int(n)
        if redraw is not None and self.redraw is not None:
            self.redraw = redraw
        assert n <= self.n_local
        if not hashes.is_cuda:
            import torch.distributed as dist
            sh, sp, sc = segment_buckets(hashes.numpy().view(np.uint64)[: 2 * n],
                                         panels.numpy().view(np.uint64)[: n * self.W].reshape(n, self.W),
                                         self.world, self.cap)
            rh, rp, rc = (torch.empty(x.shape, dtype=torch.int64) for x in (sh, sp, sc))
            dist.all_to_all_single(rc, torch.from_numpy(sc))
            dist.all_to_all_single(rh, torch.from_numpy(sh.view(np.int64)))
            dist.all_to_all_single(rp, torch.from_numpy(sp.view(np.int64)))
            u = distinct_segments(rh.numpy().view(np.uint64), rp.numpy().view(np.uint64), rc.numpy())
            return torch.tensor([u], dtype=torch.int64)
        from . import _native as N
        assert status is not None, "the device exchange reports a full segment in the status block"
        st = stream or torch.cuda.current_stream(hashes.device)
        sp_ = ctypes.c_void_p(st.cuda_stream)
        L = N.lib()
        if self.redraw is not None:
            handle, k, seed, max_att = self.redraw
            N.check(L.csa_exchange_keys_async(N.ptr(hashes), N.ptr(panels), n, self.W, int(panel_begin), self.world,
                                              self.cap, N.ptr(self.scratch), self.scratch.numel() * 8,
                                              N.ptr(self.send_k), N.ptr(self.send_c), N.ptr(status), sp_))
            with torch.cuda.stream(st):
                _all_to_all(self.recv_c, self.send_c)
                _all_to_all(self.recv_k, self.send_k)
                self.unique.zero_()
            N.check(L.csa_unique_keys_async(handle, int(k), int(seed) & M64, int(max_att), N.ptr(self.recv_k),
                                            self.world, self.cap, N.ptr(self.recv_c), N.ptr(self.owner_scratch),
                                            self.owner_scratch.numel() * 8, N.ptr(self.unique), N.ptr(status), sp_))
            with torch.cuda.stream(st):
                return self.unique.clone()
        N.check(L.csa_exchange_pack_async(N.ptr(hashes), N.ptr(panels), n, self.W, self.world, self.cap,
                                          N.ptr(self.scratch), self.scratch.numel() * 8, N.ptr(self.send_h),
                                          N.ptr(self.send_p), N.ptr(self.send_c), N.ptr(status), sp_))
        with torch.cuda.stream(st):
            _all_to_all(self.recv_c, self.send_c)
            _all_to_all(self.recv_h, self.send_h)
            _all_to_all(self.recv_p, self.send_p)
            self.table.count.zero_()
        N.check(L.csa_unique_segments_async(N.ptr(self.recv_h), N.ptr(self.recv_p), self.world, self.cap,
                                            N.ptr(self.recv_c), self.W, N.ptr(self.table.table), self.table.slots,
                                            N.ptr(self.table.count), N.ptr(status), sp_))
        with torch.cuda.stream(st):
            return self.table.count.clone()


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


def _all_reduce(t, op=None):
    import torch.distributed as dist
    op = dist.ReduceOp.SUM if op is None else op
    if _host_collectives(t):
        h = t.cpu()
        dist.all_reduce(h, op=op)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op)


def combine(counts, pairs, hashes, panels, W, exchange=None, stream=None, pair_bound=None, status=None, redraw=None,
            panel_begin=0):
    """Exchange steps for this rank; returns (counts, pairs, unique_tensor), all stream-ordered.

    counts int64[n], pairs int64[n*n] or None, hashes int64[2*S_local] and panels
    int64[S_local*W] (this rank's panels, global indices from ``panel_begin``).  Counts and pairs:
    all_reduce(SUM).  Distinct panels: ``exchange`` (a PanelExchange, built here if None, with
    ``redraw`` for the 24-byte keys) sends the local distinct panels to their owners, each owner
    counts exactly, all_reduce(SUM) of the counts.
    """
    import torch
    import torch.distributed as dist
    n_local = hashes.numel() // 2
    if exchange is None:
        # every rank must size its segments alike (equal-split all_to_all): the largest shard's
        n_max = torch.tensor([n_local], dtype=torch.int64, device=hashes.device)
        _all_reduce(n_max, op=dist.ReduceOp.MAX)
        exchange = PanelExchange(int(n_max.item()), W, dist.get_world_size(), hashes.device, redraw=redraw)
    _all_reduce(counts)
    if pairs is not None:
        _all_reduce_pairs(pairs, pair_bound, stream)
    u = exchange.run(hashes, panels, n_local, status=status, stream=stream, panel_begin=panel_begin)
    if u.is_cuda:
        with torch.cuda.stream(stream or torch.cuda.current_stream(u.device)):
            _all_reduce(u)
    else:
        _all_reduce(u)
    return counts, pairs, u


def local_distinct_rows(hashes, panels, n, W, status=None, stream=None):
    """This rank's exact distinct panels (hash AND bitmask): (uint64 rows as an int64 tensor of
    count*W words on the inputs' device, count).  Device inputs: csa_exchange_pack_async with one
    owner (the partitioned dedupe + bucketing of the exchange); host inputs: local_distinct."""
    import torch
    n, W = int(n), int(W)
    if not hashes.is_cuda:
        _, p = local_distinct(hashes.numpy().view(np.uint64)[: 2 * n], panels.numpy().view(np.uint64)[: n * W]
                              .reshape(n, W))
        return torch.from_numpy(np.ascontiguousarray(p).view(np.int64).reshape(-1)), len(p)
    from . import _native as N
    dev = hashes.device
    st = stream or torch.cuda.current_stream(dev)
    m = max(n, 1)
    send_h = torch.empty(2 * m, dtype=torch.int64, device=dev)
    send_p = torch.empty(m * W, dtype=torch.int64, device=dev)
    send_c = torch.zeros(1, dtype=torch.int64, device=dev)
    sb = int(N.lib().csa_exchange_scratch_bytes(m))
    scratch = torch.empty((sb + 7) // 8, dtype=torch.int64, device=dev)
    own_status = status if status is not None else torch.zeros(4, dtype=torch.int32, device=dev)
    N.check(N.lib().csa_exchange_pack_async(N.ptr(hashes), N.ptr(panels), n, W, 1, m, N.ptr(scratch), sb,
                                            N.ptr(send_h), N.ptr(send_p), N.ptr(send_c), N.ptr(own_status),
                                            ctypes.c_void_p(st.cuda_stream)))
    st.synchronize()
    if status is None:
        h = own_status.cpu().numpy().astype(np.uint32)
        N.check(N.lib().csa_status_decode(N.ptr(h)))
    cnt = int(send_c.item())
    return send_p[: cnt * W], cnt


class PanelRedraw:
    """found_panels of a sharded run, re-made where they are read instead of gathered.

    Every panel is a pure function of (instance, k, seed, global panel index): the Philox counter
    of each draw is (step, attempt, panel) under the key ``seed``, so the
    panels [0, S) of the whole job -- every rank's shard -- can be drawn again on any one process.
    Calling this re-draws them in chunks of ``chunk`` panels through ``draw(begin, count)`` (a
    callable returning uint64[count, W]; ``device_redraw`` for the product path) into one host
    array, with no collective: any rank may iterate, test membership or pickle its found_panels at
    any time, alone.  The reference only ever takes len() of the set (analysis.py:575, 580) and
    pickles it (analysis.py:290); len() needs no re-draw (the exchange's exact count)."""

    def __init__(self, draw, S, W, chunk=1 << 20):
        self.draw, self.S, self.W, self.chunk = draw, int(S), int(W), max(1, int(chunk))

    def __call__(self):
        out = np.empty((self.S, max(self.W, 1)), np.uint64)
        for off in range(0, self.S, self.chunk):
            c = min(self.chunk, self.S - off)
            out[off:off + c] = self.draw(off, c)
        return out


def device_redraw(enc, k, seed, device, max_attempts=0):
    """``draw(begin, count)`` for PanelRedraw on ``device``: csa_redraw_async (the batch draw's kernel
    and Philox counters, not counted in the instance's draw statistics) into a device buffer, then one
    copy to the host.  The re-drawn status block is decoded: the original call already succeeded on
    every rank, so an error here is raised, never ignored."""
    import torch
    from . import _native as N
    W = enc.W
    seed64 = int(seed) & M64

    def draw(begin, count):
        with torch.cuda.device(device):
            st = torch.cuda.current_stream(device)
            buf = torch.empty(max(count * W, 1), dtype=torch.int64, device=device)
            status = torch.zeros(4, dtype=torch.int32, device=device)
            N.check(N.lib().csa_redraw_async(enc.handle, int(k), seed64, int(begin), int(count), int(max_attempts),
                                             N.ptr(buf), N.ptr(status), ctypes.c_void_p(st.cuda_stream)))
            host = buf[:count * W].cpu()
            words = status.cpu().numpy().astype(np.uint32)
        if words[0]:
            _decode_status(words, int(words[0]))
        return host.numpy().view(np.uint64).reshape(count, W)

    return draw


ERR_DRAW_PRIORITY = 1 << 16     # status codes are small; draw errors reduce above every other code


def _decode_status(words, reduced_code):
    """Raise the error of a status block (host uint32[4]); a rank whose own block is clean -- or holds
    another error than the one the ranks agreed on (``reduced_code``) -- raises the agreed code
    (KeyError for a missing candidate, legacy.py:188), so every rank raises the same error."""
    from . import _native as N
    h = np.asarray(words, np.uint32)
    if int(h[0]) != int(reduced_code):
        h = np.array([reduced_code, 0xFFFFFFFF, 0xFFFFFFFF, 0], np.uint32)
    rc = N.lib().csa_status_decode(N.ptr(h))
    if rc == N.CSA_E_NO_CANDIDATE:
        raise KeyError("")
    N.check(rc)


def _shard_exchange(enc, n_max, world, dev):
    """The encoding's cached PanelExchange (24-byte keys) for shares of at most n_max panels."""
    ex = getattr(enc, "_xchg", None)
    if ex is None or ex.n_local < max(int(n_max), 1) or ex.world != int(world) or ex.device != dev:
        enc._xchg = None
        ex = enc._xchg = PanelExchange(n_max, enc.W, world, dev, redraw=(enc.handle, 0, 0, 0))
    return ex


def shard_device():
    """The GPU of this rank: LOCAL_RANK (one process per GPU, as torchrun sets it), modulo the visible
    devices so rehearsals can put several ranks on one GPU; without LOCAL_RANK, the current device.
    Never changes the caller's current device."""
    import torch
    lr = os.environ.get("LOCAL_RANK")
    idx = int(lr) % max(torch.cuda.device_count(), 1) if lr is not None else torch.cuda.current_device()
    return torch.device("cuda", idx)


def legacy_probabilities_distributed(instance, iterations, random_seed, keep_panels=True, chunk=None,
                                     timings=None):
    """analysis.py:162-191 with the panels sharded over the ranks of the default group.  Every rank
    returns the whole job's alloc, pair histogram and exact distinct-panel count.

    Per call (cheap when repeated): the encoding, the device pipeline (picks / XT / pair scratch
    sized to one ``chunk`` of panels, default 2^20 or CSA_SHARD_CHUNK) and the 24-byte key exchange
    are cached on the encoding; the share's panels and hashes and the n*n pair matrix are fresh
    tensors (caching allocator).  Draws, counting, pairs, the draw statistics and every collective
    are stream-ordered; the host waits once, for one copy of [counts | statistics | distinct count |
    status].  The pair counts stay on the device behind the returned PairHistogram (packed and
    divided there when first read).  Runs on ``shard_device()`` without changing the caller's current
    device.

    found_panels: len() is the exchange's exact global count.  With more than one rank (or a forced
    exchange) nothing else is kept and nothing is sent: iterating, ``in``, ``rows()`` or pickling on
    ANY rank re-draws the job's panels [0, S) on that rank's GPU (PanelRedraw, csa_redraw_async) and
    deduplicates them there -- no collective, so a rank may do it alone, at any time.  One rank (no
    exchange): the panels of the call are the whole run's and stay on the device, decoded when read, as
    the one-GPU call does.  ``keep_panels=False``: len() only.  The draw statistics
    (analysis.LAST_RUN_STATS) are summed over ranks.  ``timings`` (a dict) gets the host-side stage
    times in ms."""
    import time
    import torch
    import torch.distributed as dist
    from . import analysis as A
    from . import _native as N
    t0 = time.perf_counter()
    world, r = world_size(), rank()
    S = int(iterations)
    A.seed(random_seed)
    A.STREAM.take_panels(S)
    enc = A.encode_cached(instance.categories, instance.agents)
    k = int(instance.k)
    enc.check_quotas(k)
    begin, end = shard_range(S, world, r)
    local = end - begin
    n_max = shard_range(S, world, 0)[1]          # rank 0 holds the largest share
    dev = shard_device()
    with torch.cuda.device(dev):
        out = _sharded_call(A, N, dist, enc, k, S, random_seed, world, begin, local, n_max, dev, keep_panels, chunk,
                            t0, timings, instance)
    return out


def _sharded_call(A, N, dist, enc, k, S, random_seed, world, begin, local, n_max, dev, keep_panels, chunk, t0, timings,
                  instance):
    import time
    import torch
    C = max(1, min(max(local, 1), int(chunk or os.environ.get("CSA_SHARD_CHUNK", 1 << 20))))
    pipe = A.cached_pipeline(enc, k, C)
    # (CSA_FORCE_EXCHANGE=1: the key exchange even for one rank -- tests of its collectives on one GPU)
    ex = _shard_exchange(enc, n_max, world, dev) if world > 1 or os.environ.get("CSA_FORCE_EXCHANGE") == "1" else None
    W, n = enc.W, enc.n
    L = N.lib()
    st = pipe.stream
    sp = ctypes.c_void_p(st.cuda_stream)
    t1 = time.perf_counter()
    with torch.cuda.stream(st):
        panels = torch.empty(max(local * W, 1), dtype=torch.int64, device=dev)
        hashes = torch.empty(max(2 * local, 2), dtype=torch.int64, device=dev)
        pairs = torch.empty(n * n, dtype=torch.int64, device=dev)
        # [counts (n) | attempts, SelectionErrors, rejections | distinct count]: one all_reduce(SUM)
        acc = torch.zeros(n + 4, dtype=torch.int64, device=dev)
        pipe.reset(pairs=False)
        A.reset_draw_stats(enc, st)
        if ex is None:  # one rank: its distinct-count table before the draws (see below)
            table = getattr(enc, "_table", None)
            if table is None or table.device != dev:
                table = enc._table = HashTable(local, dev)
            table.ensure(local)
        own_counts, own_pairs = pipe.counts, pipe.pairs
        pipe.counts, pipe.pairs = acc[:n], pairs
        try:
            if local:
                pipe.draw_count_chunks(random_seed, begin, local, panels, hashes, C, overwrite_pairs=True,
                                       reset_counts=True)
            else:
                pairs.zero_()
        finally:
            pipe.counts, pipe.pairs = own_counts, own_pairs
        # this shard's draw statistics, before the exchange's re-draws (device, no host wait)
        N.check(L.csa_instance_draw_stats_async(enc.handle, N.ptr(acc[n:n + 3]), sp))
        if ex is not None:
            # a shard whose draw failed still enters the collectives (every rank must, or the others
            # hang); its status block joins the MAX all_reduce below, so every rank raises the draw's
            # error -- the exchange writes its own status only past a full segment, and the first
            # error recorded in a block wins (csa_status_decode)
            _all_reduce_pairs(pairs, S, st)
            u = ex.run(hashes, panels, local, status=pipe.status, stream=st, panel_begin=begin,
                       redraw=(enc.handle, k, random_seed, 0))
        else:
            # one rank owns every panel: nothing to reduce, and the exact local distinct count runs on
            # a side stream after the draws, beside the last chunk's counting and pairs (as
            # analysis.legacy_sample_device; the table was allocated before the draws were enqueued)
            ust = getattr(pipe, "unique_stream", None)
            if ust is None:
                ust = pipe.unique_stream = torch.cuda.Stream(dev)
            ust.wait_stream(pipe.draw_stream if local else st)
            with torch.cuda.stream(ust):
                table.count.zero_()
                N.check(L.csa_unique_async(N.ptr(hashes), N.ptr(panels), local, W, N.ptr(table.table),
                                           table.slots, N.ptr(table.count), N.ptr(pipe.status),
                                           ctypes.c_void_p(ust.cuda_stream)))
            st.wait_stream(ust)
            u = table.count
        acc[n + 3:].copy_(u)
        code = pipe.status[:1].to(torch.int64)
        if ex is not None:
            _all_reduce(acc)
            # MAX over ranks of a priority key: a draw error (KeyError / attempt limit) on any rank
            # outranks an exchange error on another (an overflowing segment), whatever their codes
            code += ERR_DRAW_PRIORITY * ((code == N.CSA_E_NO_CANDIDATE) | (code == N.CSA_E_ATTEMPT_LIMIT))
            _all_reduce(code, op=dist.ReduceOp.MAX)
            code %= ERR_DRAW_PRIORITY
        tail = torch.cat([code, pipe.status.to(torch.int64)])
        host = torch.cat([acc, tail]).cpu()          # the call's one host wait
    t2 = time.perf_counter()
    h = host.numpy()
    if int(h[n + 4]):
        _decode_status((h[n + 5:n + 9] & 0xFFFFFFFF).astype(np.uint32), int(h[n + 4]))
    counts = h[:n].copy()
    stats = dict(zip(A.STAT_KEYS, (int(x) for x in h[n:n + 3])))
    # one rank (no exchange): its panels are the whole run's, so found_panels keeps them on the device and
    # decodes them when iterated, as the one-GPU call does
    solo = ex is None and keep_panels
    raw = A.LegacyRaw(counts, pairs.view(n, n), int(h[n + 3]), panels[: local * W] if solo else None, None, stats)
    out = A.finish(instance, enc, raw, S)
    if keep_panels and not solo:
        # nothing kept, nothing sent: the whole job's panels are re-drawn where they are read
        out[1]._redraw = PanelRedraw(device_redraw(enc, k, random_seed, dev), S, W, chunk=max(C, 1 << 16))
    if timings is not None:
        t3 = time.perf_counter()
        timings.update(setup_ms=(t1 - t0) * 1e3, device_ms=(t2 - t1) * 1e3, finish_ms=(t3 - t2) * 1e3,
                       total_ms=(t3 - t0) * 1e3)
    return out
