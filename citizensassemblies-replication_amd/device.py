"""Device-resident LEGACY pipeline on one GPU (stream-ordered C ABI + torch buffers).

PyTorch only provides device memory, the stream and (in distributed.py) the
RCCL collectives; every kernel is the hand-written HIP in csrc/.  One
``run`` = one pass of analysis.py:162-191 over a shard of panels:

    draw_lane_kernel   panels [panel_begin, panel_begin+S) -> pick lists, then (in the same
                       kernel, per workgroup) packed bitmasks + 128-bit panel hashes   (draw)
    picks_pack_kernel  pick lists -> bitmasks + hashes for the wide kernel, or after
                       draw_picks (the split form, kept for A/B)                        (pack)
      (instances beyond both: draw_kernel writes bitmasks + hashes directly)
    xt_count_kernel    bitmasks -> transposed panel-indicator bits + per-person counts (+=)
    pair_mfma_kernel   transposed bits -> int32 partial blocks of X^T X on fp4 (default) or
    pair_reduce_kernel   int8 MFMA -> pair counts (+=, or = with overwrite)  (if want_pairs)
    uq_* kernels       hashes + bitmasks -> exact distinct-panel count (+=) (if want_unique)

Buffers are allocated once for the largest shard and reused across runs, so a
timed loop measures kernels only.
"""
import ctypes

import torch

from . import _native as N


def _stream_ptr(stream):
    return ctypes.c_void_p(stream.cuda_stream) if stream is not None else None


def chunk_plan(S, C, R):
    """Chunk sizes (summing to S, each <= C) for DevicePipeline.draw_count_chunks.  R > 0 is the
    draw's round (csa_draw_round_panels): every chunk but the last is a whole number of rounds, so
    no launch but the last ends in a part-empty round of waves, and the last two are one round and
    the remainder, so the counting of the big chunk runs beside two short draws and only the
    remainder's counting follows the last draw.  R = 0: equal cuts of at most C (flat)."""
    S, C = int(S), max(1, int(C))
    if S <= 0:
        return []
    if R <= 0 or S <= R or R > C:
        return [min(C, S - off) for off in range(0, S, C)]
    tail = S - R * ((S - 1) // R)                 # in (0, R]
    head = S - tail - R                           # whole rounds before the last full one
    Cr = (C // R) * R
    sizes = []
    while head > 0:
        c = min(Cr, head)
        sizes.append(c)
        head -= c
    return sizes + [R, tail]


class DevicePipeline:
    def __init__(self, enc, k, max_panels, want_pairs=True, want_unique=True, want_attempts=False,
                 device=None, stream=None, pair_engine=N.CSA_PAIR_FP4, pairs_buffer=True):
        """``pairs_buffer=False``: no n*n pair matrix of its own (the caller sets ``self.pairs``
        before ``pair_counts``); XT and the pair scratch are still allocated with want_pairs."""
        self.enc = enc
        self.k = int(k)
        self.device = torch.device(device or "cuda")
        self.stream = stream or torch.cuda.current_stream(self.device)
        self.want_pairs = want_pairs
        self.want_unique = want_unique
        self.pair_engine = int(pair_engine)
        S = int(max_panels)
        self.max_panels = S
        n, W = enc.n, enc.W
        L = N.lib()
        self.npad = int(L.csa_xt_pad(max(n, 1)))
        nblk = (S + 63) // 64
        slots = 1
        while slots < max(2 * S, 64):
            slots <<= 1
        self.slots = slots
        dev = self.device
        u64 = torch.int64  # raw 64-bit words; reinterpretation is done by the kernels
        with torch.cuda.device(dev):
            _ = enc.handle  # upload the instance on this device
            # the lane kernel writes pick lists (u16) that picks_pack_kernel packs; others write bitmasks
            self.split_draw = bool(L.csa_draw_picks_supported(enc.handle, self.k)) and self.k > 0
            self.kpad = int(L.csa_picks_stride(self.k))
            self.picks = torch.empty(max(S * self.kpad, 1), dtype=torch.int16, device=dev) if self.split_draw else None
            self.panels = torch.empty(S * W, dtype=u64, device=dev)
            self.hashes = torch.empty(2 * S, dtype=u64, device=dev) if want_unique else None
            self.attempts = torch.empty(S, dtype=torch.int32, device=dev) if want_attempts else None
            self.status = torch.zeros(4, dtype=torch.int32, device=dev)
            self.counts = torch.zeros(n, dtype=torch.int64, device=dev)
            self.xt = torch.empty(nblk * self.npad, dtype=u64, device=dev) if want_pairs else None
            self.pairs = torch.zeros(n * n, dtype=torch.int64, device=dev) if want_pairs and pairs_buffer else None
            sb = int(L.csa_pair_scratch_bytes(max(n, 1), max(nblk, 1), self.pair_engine)) if want_pairs else 0
            self.pair_scratch = torch.empty((sb + 3) // 4, dtype=torch.int32, device=dev) if want_pairs else None
            self.table = torch.empty(slots, dtype=u64, device=dev) if want_unique else None
            self.unique = torch.zeros(1, dtype=torch.int64, device=dev)

    def reset(self, status=True, pairs=True, counts=True):
        """Zero the accumulators.  ``pairs=False`` skips the n*n pair matrix for a caller whose next
        ``pair_counts(..., overwrite=True)`` stores the batch's counts instead of adding them;
        ``counts=False`` leaves the counts and the distinct count (draw_count_chunks(reset_counts=True)
        zeroes the counts after the draws are enqueued)."""
        with torch.cuda.stream(self.stream):
            if status:
                self.status.zero_()
            if counts:
                self.counts.zero_()
                self.unique.zero_()
            if pairs and self.pairs is not None:
                self.pairs.zero_()

    # individual stages (stream-ordered, no sync) -------------------------------------------
    def draw_picks(self, seed, panel_begin, S, max_attempts=0, stream=None):
        """Pick-list draw (draw_lane_kernel) into self.picks; ``pack`` turns it into panels."""
        assert self.split_draw and S <= self.max_panels
        N.check(N.lib().csa_draw_picks_async(self.enc.handle, self.k, int(seed) & 0xFFFFFFFFFFFFFFFF,
                                             int(panel_begin), int(S), max_attempts, N.ptr(self.picks),
                                             N.ptr(self.attempts), N.ptr(self.status),
                                             _stream_ptr(stream or self.stream)))

    def pack(self, S, stream=None):
        """Pick lists -> self.panels (+ self.hashes with want_unique)."""
        N.check(N.lib().csa_picks_pack_async(N.ptr(self.picks), int(S), self.k, self.enc.n, N.ptr(self.panels),
                                             N.ptr(self.hashes), _stream_ptr(stream or self.stream)))

    def draw(self, seed, panel_begin, S, max_attempts=0, stream=None):
        """Draw into self.panels (and, with want_unique, their hashes into self.hashes) on
        ``stream`` (default: the pipeline's stream).  A caller that overlaps the draw of the next
        batch with this batch's counting swaps ``self.panels`` / ``self.hashes`` between buffers
        and orders the streams with events (bench.py)."""
        assert S <= self.max_panels and self.panels.numel() >= S * self.enc.W
        # lane-kernel instances pack their panels inside the draw kernel (fused); the wide kernel's
        # pick lists are packed by picks_pack_kernel inside the same call
        N.check(N.lib().csa_draw_async(self.enc.handle, self.k, int(seed) & 0xFFFFFFFFFFFFFFFF, int(panel_begin),
                                       int(S), max_attempts, N.ptr(self.panels), N.ptr(self.hashes),
                                       N.ptr(self.attempts), None, N.ptr(self.status),
                                       _stream_ptr(stream or self.stream)))

    def draw_xt(self, seed, panel_begin, S, max_attempts=0, reset=False, stream=None):
        """draw() on ``stream`` (default: the pipeline's stream) that also writes the panels as XT into
        self.xt when the instance takes a register kernel with a fused pack (draw_lane_kernel /
        draw_solo_kernel; csa_draw_xt_async).  Returns True when it did: the caller then skips
        transpose_count and takes the counts from the pair diagonal (counts_from_pairs).  ``reset``: the
        status words and the instance's draw statistics are zeroed first, in the same call
        (stream-ordered).  A caller that overlaps draws with counting swaps ``self.xt`` between
        buffers like ``self.panels`` (bench.py)."""
        assert S <= self.max_panels and self.panels.numel() >= S * self.enc.W and self.want_pairs
        written = ctypes.c_int32(0)
        N.check(N.lib().csa_draw_xt_async(self.enc.handle, self.k, int(seed) & 0xFFFFFFFFFFFFFFFF, int(panel_begin),
                                          int(S), max_attempts, N.ptr(self.panels), N.ptr(self.hashes),
                                          N.ptr(self.attempts), N.ptr(self.status), N.ptr(self.xt),
                                          ctypes.byref(written),
                                          (N.CSA_DRAW_RESET_STATUS | N.CSA_DRAW_RESET_STATS) if reset else 0,
                                          _stream_ptr(stream or self.stream)))
        return bool(written.value)

    def counts_from_pairs(self):
        """self.counts = the diagonal of self.pairs (stored; after pair_counts of the whole batch)."""
        N.check(N.lib().csa_pairs_diag_async(N.ptr(self.pairs), self.enc.n, N.ptr(self.counts),
                                             _stream_ptr(self.stream)))

    def hash(self, S):
        N.check(N.lib().csa_panel_hash_async(N.ptr(self.panels), int(S), self.enc.W, N.ptr(self.hashes),
                                             _stream_ptr(self.stream)))

    def draw_kernel_name(self):
        buf = ctypes.create_string_buffer(128)
        N.check(N.lib().csa_draw_kernel_name(self.enc.handle, self.k, buf, 128))
        return buf.value.decode()

    def transpose_count(self, S):
        N.check(N.lib().csa_transpose_count_async(N.ptr(self.panels), int(S), self.enc.n,
                                                  N.ptr(self.xt) if self.want_pairs else None,
                                                  N.ptr(self.counts), _stream_ptr(self.stream)))

    def pair_counts(self, S, overwrite=False, shared=False, alone=False):
        """Pair counts of the batch into self.pairs: added (default) or, with ``overwrite``, stored
        (upper triangle incl. the diagonal; CSA_PAIR_OVERWRITE, no zero-fill needed).  ``shared``:
        the launch overlaps draws on another stream (CSA_PAIR_SHARED, a scheduling hint); ``alone``:
        no draw runs beside it (CSA_PAIR_ALONE: the kernel fastest alone)."""
        nblk = (int(S) + 63) // 64
        L = N.lib()
        need = int(L.csa_pair_scratch_bytes(self.enc.n, nblk, self.pair_engine))
        assert need <= self.pair_scratch.numel() * 4
        N.check(L.csa_pair_counts_ex_async(N.ptr(self.xt), nblk, self.enc.n, N.ptr(self.pairs),
                                           self.pair_engine | (N.CSA_PAIR_OVERWRITE if overwrite else 0)
                                           | (N.CSA_PAIR_SHARED if shared else 0)
                                           | (N.CSA_PAIR_ALONE if alone else 0),
                                           N.ptr(self.pair_scratch), self.pair_scratch.numel() * 4,
                                           _stream_ptr(self.stream)))

    def unique_count(self, S):
        N.check(N.lib().csa_unique_async(N.ptr(self.hashes), N.ptr(self.panels), int(S), self.enc.W,
                                         N.ptr(self.table), self.slots, N.ptr(self.unique), N.ptr(self.status),
                                         _stream_ptr(self.stream)))

    def round_panels(self):
        """Panels one full round of the batch draw's resident workgroups covers on this device
        (csa_draw_round_panels; 131072 for the two-lane kernel on 256 CUs)."""
        rp = getattr(self, "_round", None)
        if rp is None:
            import numpy as np
            out = np.zeros(1, np.uint64)
            N.check(N.lib().csa_draw_round_panels(self.enc.handle, self.k, N.ptr(out)))
            rp = self._round = max(1, int(out[0]))
        return rp

    def draw_count_chunks(self, seed, panel_begin, S, panels, hashes, chunk, overwrite_pairs=False,
                          reset_counts=False):
        """Draw S panels (global indices panel_begin ..) into ``panels`` / ``hashes`` (tensors of the
        whole batch) and accumulate their counts and pairs, in chunks of at most ``chunk`` panels
        (at most max_panels): every chunk's draw is enqueued at once on the pipeline's draw stream, each into
        its own slice, and the pipeline stream counts and pairs chunk c after chunk c's draw event --
        beside the draw of chunk c + 1 (bench.py's pipeline).  The first chunk stores its pair counts
        with ``overwrite_pairs``; later chunks add theirs.  Ordered after everything already on the
        pipeline stream; on return the pipeline stream is ordered after every draw.  ``reset_counts``:
        the per-person counts are zeroed on the pipeline stream after the draws are enqueued (before
        the first chunk's counting), so the draws do not wait for it.  With ``overwrite_pairs`` and
        ``reset_counts`` on an instance whose draw writes XT itself (xt_fused), the chunks take
        _draw_xt_chunks instead: no transpose pass, the counts from the pair diagonal."""
        import os
        import torch
        S, C, W = int(S), max(1, min(int(chunk), self.max_panels)), self.enc.W
        # flat cuts by default: the round-aligned plan (CSA_CHUNK_PLAN=round) measured slower end to end
        # (sf_e 10^6 panels 4.59 vs 4.41 ms, example_large_200 1.25e6 5.02 vs 4.99, synthetic8192 10^6
        # 33.0 vs 32.2; profiles/r05_api_chunk_plan.txt): the big chunk's counting slows the short draws
        sizes = chunk_plan(S, C, self.round_panels() if os.environ.get("CSA_CHUNK_PLAN") == "round" else 0)
        chunks, off = [], 0
        for ln in sizes:
            chunks.append((off, ln))
            off += ln
        st = getattr(self, "draw_stream", None)
        if st is None:
            st = self.draw_stream = torch.cuda.Stream(self.device)
        st.wait_stream(self.stream)
        if chunks and self.want_pairs and overwrite_pairs and reset_counts and self.xt_fused() and \
                os.environ.get("CSA_DRAW_XT", "1") != "0":
            return self._draw_xt_chunks(seed, panel_begin, panels, hashes, chunks, st)
        own_p, own_h = self.panels, self.hashes
        try:
            drawn = []
            for off, ln in chunks:
                self.panels, self.hashes = panels[off * W:(off + ln) * W], hashes[2 * off:2 * (off + ln)]
                self.draw(seed, panel_begin + off, ln, stream=st)
                ev = torch.cuda.Event()
                ev.record(st)
                drawn.append(ev)
            if reset_counts:
                with torch.cuda.stream(self.stream):
                    self.counts.zero_()
            for j, (off, ln) in enumerate(chunks):
                self.stream.wait_event(drawn[j])
                self.panels = panels[off * W:(off + ln) * W]
                self.transpose_count(ln)
                if self.want_pairs:
                    # the last chunk's pairs run after every draw of the call: the kernel fastest alone
                    self.pair_counts(ln, overwrite=overwrite_pairs and j == 0, shared=j + 1 < len(chunks),
                                     alone=j + 1 == len(chunks))
        finally:
            self.panels, self.hashes = own_p, own_h

    def xt_fused(self):
        """True when this instance's batch draw is a register kernel with a fused pack (draw_lane_kernel /
        draw_solo_kernel), i.e. draw_xt can write the XT operand itself."""
        f = getattr(self, "_xt_fused", None)
        if f is None:
            f = self._xt_fused = self.want_pairs and self.draw_kernel_name().startswith(("draw_lane", "draw_solo"))
        return f

    XT_RING = 3   # XT buffers of draw_count_chunks' fused form (the draw of chunk c reuses chunk c - 3's)

    def _draw_xt_chunks(self, seed, panel_begin, panels, hashes, chunks, st):
        """draw_count_chunks for instances whose draw writes XT (csa_draw_xt_async): chunk c's draw, on the
        draw stream, writes its panels, hashes and XT (a ring of XT_RING buffers: the draw of chunk c waits
        for the pairs of chunk c - XT_RING, which ran long before), and the pipeline stream runs only the
        pair kernel of chunk c after its draw (stored for the first chunk, added after); the counts are the
        pair matrix's diagonal at the end (stored) -- no transpose pass (csa_transpose_count_async)."""
        import torch
        W = self.enc.W
        ring = getattr(self, "_xt_ring", None)
        if ring is None or ring[0].numel() != self.xt.numel():
            ring = self._xt_ring = [self.xt] + [torch.empty_like(self.xt) for _ in range(self.XT_RING - 1)]
        own_p, own_h, own_xt = self.panels, self.hashes, self.xt
        drawn, counted, fused = [], [], []
        try:
            def count(j):
                off, ln = chunks[j]
                self.stream.wait_event(drawn[j])
                self.panels, self.xt = panels[off * W:(off + ln) * W], ring[j % len(ring)]
                if not fused[j]:                       # (not expected: xt_fused() said the draw writes XT)
                    self.transpose_count(ln)
                self.pair_counts(ln, overwrite=j == 0, shared=j + 1 < len(chunks), alone=j + 1 == len(chunks))
                ev = torch.cuda.Event()
                ev.record(self.stream)
                counted.append(ev)

            for j, (off, ln) in enumerate(chunks):
                if j >= len(ring):
                    st.wait_event(counted[j - len(ring)])   # that chunk's pairs have read this XT buffer
                self.panels, self.hashes = panels[off * W:(off + ln) * W], hashes[2 * off:2 * (off + ln)]
                self.xt = ring[j % len(ring)]
                fused.append(self.draw_xt(seed, panel_begin + off, ln, stream=st))
                ev = torch.cuda.Event()
                ev.record(st)
                drawn.append(ev)
                if j:
                    count(j - 1)
            count(len(chunks) - 1)
            self.counts_from_pairs()
        finally:
            self.panels, self.hashes, self.xt = own_p, own_h, own_xt

    def run(self, seed, panel_begin, S, max_attempts=0, overwrite_pairs=False):
        """Enqueue the whole pass; results accumulate into counts / pairs / unique (pairs are
        stored instead with ``overwrite_pairs``)."""
        self.draw(seed, panel_begin, S, max_attempts)
        self.transpose_count(S)
        if self.want_pairs:
            self.pair_counts(S, overwrite=overwrite_pairs)
        if self.want_unique:
            self.unique_count(S)

    def check_status(self):
        """Synchronise and raise on a device-side error (no-candidate, attempt limit)."""
        self.stream.synchronize()
        h = self.status.cpu().numpy().astype("uint32")
        rc = N.lib().csa_status_decode(N.ptr(h))
        if rc == N.CSA_E_NO_CANDIDATE:
            raise KeyError("")       # legacy.py:188
        N.check(rc)

    def panels_view(self, S):
        """Host copy of the packed panels (uint64[S, W])."""
        import numpy as np
        return self.panels[: S * self.enc.W].cpu().numpy().view(np.uint64).reshape(S, self.enc.W)
