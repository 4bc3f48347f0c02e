"""Drop-in for the LEGACY part of the reference's analysis.py, backed by HIP kernels.

Kept names and semantics (reference file:line):
  * ``Instance``, ``read_instance``    analysis.py:54-58, 108-138 (from .instance)
  * ``PairHistogram``                  analysis.py:68-98 -- same methods, backed by one
                                       packed array of the n(n-1)/2 pair values (row-major
                                       i < j) instead of a dict, filled on the device
  * ``legacy_find``                    analysis.py:141-159 -- restarts run on the device
  * ``legacy_probabilities``           analysis.py:162-191 -- the batch entry point:
                                       draw S panels (each panel's state in the registers
                                       of 1, 2 or 8 lanes of a wavefront, by instance
                                       shape), per-person counts, X^T X pair counts on fp4
                                       MFMA (exact 0/1 products, f32 accumulation; int8
                                       selectable), exact distinct-panel count; returns
                                       ``(alloc, found_panels, pair_histogram)``.
LEXIMIN / XMIN and the plotting / statistics code stay in the reference (CPU).
"""
import ctypes
import os
from typing import Dict, List, Tuple

import numpy as np

from . import _native as N
from .instance import Instance, read_instance, encode, encode_cached, unpack_panel  # noqa: F401
from . import legacy as _legacy
from .legacy import STREAM, seed, SelectionError, check_min_cats, mt_draw  # noqa: F401


def __getattr__(name):           # analysis.RNG_MODE follows legacy.RNG_MODE (set_rng_mode)
    if name == "RNG_MODE":
        return _legacy.RNG_MODE
    raise AttributeError(name)

ProbAllocation = Dict


def _divide(u, d):
    """u / d as the reference's `/` on every value (analysis.py:86-88): numpy true division, except
    integer counts over an int that float64 cannot hold exactly, which Python divides exactly
    (int / int is correctly rounded; numpy would round the divisor first)."""
    if u.dtype.kind in "iu" and isinstance(d, (int, np.integer)) and not isinstance(d, bool) and float(d) != d:
        return np.array([x / int(d) for x in u.tolist()], np.float64)
    return u / d


class PairHistogram:
    """analysis.py:68-98 with a packed backing store.

    The reference keeps a dict of the n(n-1)/2 pairs i < j in row-major key order
    (analysis.py:70); here the same values sit in one array ``_u`` of that length and
    order (strict upper triangle, row-major: pair (i, j) at i(n-1) - i(i-1)/2 + j-i-1).
    Integer counts stay exact until
    ``turn_into_probabilities_by_dividing_all_elements_by_given_number`` divides them
    (float64 true division, as the reference's ``/``).  A histogram built by
    ``legacy_probabilities`` keeps the device's n*n integer pair counts and materialises
    ``_u`` on first access: the triangle is packed and divided on the device
    (csa_pairs_upper_async) and only its n(n-1)/2 float64 values cross PCIe, so a caller
    that only reads per-person probabilities or ``len(found_panels)`` never moves it.
    """

    def __init__(self, number_of_agents, uniform_distribution=False, counts=None):
        n = int(number_of_agents)
        self.n = n
        self._src = None        # lazily materialised integer counts: n*n numpy array or device tensor
        self._divs = []         # divisions pending on _src, applied in order at materialisation
        self._uv = None
        if counts is not None:
            if hasattr(counts, "device") and not isinstance(counts, np.ndarray):
                self._src = counts
            else:
                c = np.asarray(counts)
                assert c.shape == (n, n)
                self._src = c
        else:
            self._uv = np.zeros(n * (n - 1) // 2, np.int64)
        self._counts = self._S = None   # integer pair counts and S when built by finish()
        if uniform_distribution:
            npairs = n * (n - 1) // 2
            self._src = None
            self._uv = np.full(npairs, 1 / npairs if npairs else 0.0, np.float64)

    def _materialise_device(self):
        """Strict upper triangle of the device counts, packed (and divided by the first pending
        divisor) on the device; one n(n-1)/2 copy into pinned host memory."""
        import torch
        src, n = self._src, self.n
        m = n * (n - 1) // 2
        # the device divides only by a first divisor that is positive and exact in float64 (S, as
        # legacy_probabilities passes it); any other divisor -- negative, fractional types, huge ints --
        # is applied on the host, in order, as numpy true division
        d0 = self._divs[0] if self._divs else None
        on_device = d0 is not None and isinstance(d0, (int, float, np.integer, np.floating)) and \
            not isinstance(d0, bool) and float(d0) > 0.0 and float(d0) == d0
        div = float(d0) if on_device else 0.0
        rest = self._divs[1:] if on_device else list(self._divs)
        dt = torch.float64 if on_device else torch.int64
        dev = src.device
        with torch.cuda.device(dev):
            st = torch.cuda.current_stream(dev)
            d = torch.empty(max(m, 1), dtype=dt, device=dev)
            N.check(N.lib().csa_pairs_upper_async(N.ptr(src), n, div, N.ptr(d), ctypes.c_void_p(st.cuda_stream)))
            h = torch.empty(max(m, 1), dtype=dt, pin_memory=True)
            h.copy_(d, non_blocking=True)
            st.synchronize()
        u = h.numpy()[:m]
        for dv in rest:
            u = _divide(u, dv)
        return u

    @property
    def _u(self):
        if self._uv is None:
            if isinstance(self._src, np.ndarray):
                u = self._src[np.triu_indices(self.n, 1)]
                for d in self._divs:
                    u = _divide(u, d)
            else:
                u = self._materialise_device()
            self._uv, self._src, self._divs = u, None, []
        return self._uv

    @_u.setter
    def _u(self, value):
        self._uv, self._src, self._divs = value, None, []

    def _index(self, i, j):
        return i * (self.n - 1) - i * (i - 1) // 2 + (j - i - 1)

    # dict-compatible accessors -----------------------------------------------------------
    def _key(self, key):
        i, j = sorted(key)
        if not (0 <= i < j < self.n):
            raise KeyError(key)
        return i, j

    def __getitem__(self, key):
        i, j = self._key(key)
        return self._u[self._index(i, j)].item()

    def _writable(self, as_float):
        u = self._u
        if as_float and u.dtype.kind != "f":
            u = u.astype(np.float64)
        elif not u.flags.writeable or u.base is not None:
            u = u.copy()
        self._u = u
        return u

    def __setitem__(self, key, value):
        i, j = self._key(key)
        self._counts = self._S = None
        self._writable(isinstance(value, float))[self._index(i, j)] = value

    def turn_into_probabilities_by_dividing_all_elements_by_given_number(self, num):
        # analysis.py:86-88 divides every value with Python's `/`: a zero divisor raises
        # ZeroDivisionError at once (for int and float values alike) when there is any pair
        if num == 0 and len(self):
            raise ZeroDivisionError("division by zero")
        if self._uv is None:
            self._divs.append(num)
        else:
            self._u = _divide(self._uv, num)
        self._counts = self._S = None

    def add_portfolio_of_panels_to_histogram(self, portfolio, probabilities):
        self._counts = self._S = None
        for panel, pob in zip(portfolio, probabilities):
            idx = np.asarray(sorted(panel), np.int64)
            u = self._writable(isinstance(pob, float))
            ii, jj = np.triu_indices(len(idx), 1)
            np.add.at(u, self._index(idx[ii], idx[jj]), pob)

    def upper(self):
        """Values of all pairs i < j in the reference's key order (row-major); read-only."""
        u = self._u.view()
        u.flags.writeable = False
        return u

    def get_dict(self):
        iu = np.triu_indices(self.n, 1)
        vals = self._u.tolist()
        return dict(zip(zip(iu[0].tolist(), iu[1].tolist()), vals))

    def __len__(self):
        return self.n * (self.n - 1) // 2

    def __getstate__(self):
        return {"n": self.n, "u": np.ascontiguousarray(self._u)}

    def __setstate__(self, st):
        self.n = st["n"]
        self._src, self._divs, self._uv = None, [], st.get("u")
        if self._uv is None:                     # round-4 pickles held the n*n matrix
            self._uv = np.asarray(st["m"])[np.triu_indices(self.n, 1)]
        self._counts = self._S = None


class PanelSet:
    """Set of distinct panels (found_panels, analysis.py:171,186), lazily materialised.

    ``len()`` is the device's exact distinct-panel count; iteration / membership
    decode the packed bitmasks (host array, or a device tensor copied on first
    use) into sorted agent-id tuples, as the reference's set holds them.  A
    sharded run keeps no panels: they are re-drawn where first read (``_redraw``).
    """

    def __init__(self, unique_count, packed=None, n=0, agent_ids=None):
        self._count = int(unique_count)
        self._packed = packed
        self._n = n
        self._ids = agent_ids
        self._set = None

    def __len__(self):
        return self._count

    _where = "panels were not kept; only len() is available"
    # a sharded run (distributed.PanelRedraw): nothing was kept or sent -- the job's panels are
    # re-drawn on this process's GPU when first read, then deduplicated like kept panels
    _redraw = None

    def _panels(self):
        """The kept (or re-drawn) panels, device tensor or host array; None if none were kept."""
        if self._packed is None and self._redraw is not None:
            self._packed, self._redraw = self._redraw(), None
            self._check_count = True
        return self._packed

    def _distinct(self, p):
        """Sorted distinct rows of packed panels p; a re-drawn set must have the run's exact count."""
        if hasattr(p, "device") and not isinstance(p, np.ndarray):
            p = p.cpu().numpy()
        W = max((self._n + 63) // 64, 1)
        p = np.ascontiguousarray(p).view(np.uint64).reshape(-1, W)
        rows = np.unique(p, axis=0) if len(p) else p
        if getattr(self, "_check_count", False) and len(rows) != self._count:
            raise RuntimeError("found_panels: the re-drawn panels hold %d distinct panels, the run counted %d"
                               % (len(rows), self._count))
        return rows

    def _materialise(self):
        if self._set is None:
            if self._panels() is None:
                raise RuntimeError(self._where)
            rows = self._distinct(self._packed)
            ids = self._ids
            self._set = {tuple(ids[q] for q in unpack_panel(r, self._n)) for r in rows}
            self._packed = None
        return self._set

    def __iter__(self):
        return iter(self._materialise())

    def __contains__(self, panel):
        return tuple(panel) in self._materialise()

    def __eq__(self, other):
        return set(self) == set(other)

    def rows(self):
        """The distinct panels as a host uint64[u, W] array (sorted rows), or None when the panels
        were not kept.  Device panels are copied to the host here; a sharded run's are re-drawn."""
        W = (self._n + 63) // 64
        if self._panels() is None:
            if self._set is None:
                return None
            pos = {aid: q for q, aid in enumerate(self._ids)}
            rows = np.zeros((len(self._set), max(W, 1)), np.uint64)
            for i, panel in enumerate(self._set):
                for aid in panel:
                    q = pos[aid]
                    rows[i, q >> 6] |= np.uint64(1) << np.uint64(q & 63)
            return np.unique(rows, axis=0) if len(rows) else rows
        self._packed = self._distinct(self._packed)   # keep the host rows (a re-draw happens once)
        self._check_count = False
        return self._packed

    # pickling (run_legacy_or_retrieve dumps the returned tuple, analysis.py:284-290): only host
    # data -- the distinct panels as packed rows (or the materialised set) -- so the pickle loads
    # on a machine without a GPU
    def __getstate__(self):
        st = {"count": self._count, "n": self._n, "ids": self._ids}
        if self._set is not None:
            st["set"] = self._set
        else:
            st["rows"] = self.rows()
        return st

    def __setstate__(self, st):
        self._count, self._n, self._ids = st["count"], st["n"], st["ids"]
        self._set = st.get("set")
        self._packed = st.get("rows")


def _with_address(enc, columns_data, check_same_address_columns):
    """Same-address rings for the encoded agents (None without columns)."""
    if columns_data is None or not check_same_address_columns:
        return None
    return _legacy.address_rings(enc.agent_ids, columns_data, check_same_address_columns)


def legacy_find(feature_info, agents, k, rng: str = None, *, columns_data=None,
                check_same_address_columns=None) -> List:
    """analysis.py:141-159: one accepted panel, pick order, restarts on the device (Philox
    stream) or, with rng="mt" (default: legacy.RNG_MODE), on the host from the stdlib random
    stream as the reference consumes it.  With ``columns_data`` and
    ``check_same_address_columns`` the draws delete same-address people (legacy.py:109-113;
    the reference's legacy_find always passes check_same_address=False, analysis.py:150-151)."""
    return legacy_find_batch(feature_info, agents, k, 1, rng=rng, columns_data=columns_data,
                             check_same_address_columns=check_same_address_columns)[0]


def legacy_find_batch(feature_info, agents, k, count, max_attempts=0, rng: str = None, *, columns_data=None,
                      check_same_address_columns=None):
    """``count`` consecutive legacy_find calls in one launch (XMIN's caller, xmin.py:464-474)."""
    enc = encode_cached(feature_info, agents)
    k = int(k)
    ring = _with_address(enc, columns_data, check_same_address_columns)
    ids = enc.agent_ids
    if (rng or _legacy.RNG_MODE) == "mt":
        picks, _, _ = mt_draw(enc, k, int(count), max_attempts=max_attempts, addr_next=ring)
        return [[ids[int(p)] for p in row[:k] if p >= 0] for row in picks]
    picks = np.full((int(count), max(k, 1)), -1, np.int32)
    L = N.lib()
    first = STREAM.take_panels(count)
    if ring is not None:
        N.check(L.csa_instance_set_address(enc.handle, N.ptr(ring)))
    try:
        N.check(L.csa_legacy_find(enc.handle, k, STREAM.key, first, int(count), max_attempts, N.ptr(picks), None))
    finally:
        if ring is not None:
            N.check(L.csa_instance_set_address(enc.handle, None))
    return [[ids[int(p)] for p in row[:k] if p >= 0] for row in picks]


class LegacyRaw:
    """Integer results of one legacy_probabilities run (exact, before division).  ``stats``: the
    run's draw statistics (attempts, SelectionErrors, min-quota rejections; see draw_stats)."""

    def __init__(self, counts, pairs, unique, panels, attempts, stats=None):
        self.counts, self.pairs, self.unique, self.panels, self.attempts = counts, pairs, unique, panels, attempts
        self.stats = stats


STAT_KEYS = ("attempts", "selection_errors", "rejections")
# draw statistics of the last legacy_probabilities call (SURVEY.md section 5 "Metrics"): the
# reference prints "Rejected" per min-quota rejection (analysis.py:159) and restarts silently on a
# SelectionError (analysis.py:152-153); here both are counted on the device
LAST_RUN_STATS = None


def reset_draw_stats(enc, stream=None):
    """Zero the instance's draw statistics before a batch: ordered on ``stream`` (a torch stream the
    batch's draws run on; no host wait), or, without one, after the instance's own streams and the
    streams of the encoding's cached DevicePipeline (its draw stream included: draws a caller
    enqueued there may still be counting) are idle (csa_instance_draw_stats_reset) -- never a
    device-wide synchronisation.  A caller that drew on streams of its own (bench.py)
    synchronises them first or passes the stream."""
    if stream is None:
        pipe = getattr(enc, "_pipe", None)
        for st in (getattr(pipe, "draw_stream", None), getattr(pipe, "stream", None)):
            if st is not None:
                st.synchronize()
    N.check(N.lib().csa_instance_draw_stats_reset(enc.handle, ctypes.c_void_p(stream.cuda_stream)
                                                  if stream is not None else None))


def draw_stats(enc, reset=False):
    """Totals of the instance's draws since creation / the last reset (csa_instance_draw_stats):
    {"attempts", "selection_errors", "rejections"}.  Synchronises the device."""
    out = np.zeros(3, np.uint64)
    N.check(N.lib().csa_instance_draw_stats(enc.handle, 1 if reset else 0, N.ptr(out)))
    return dict(zip(STAT_KEYS, (int(x) for x in out)))


def legacy_sample_raw(enc, k, iterations, random_seed, panel_begin=0, want_pairs=True, want_panels=True,
                      want_attempts=False, max_attempts=0, devices=None):
    """Run the whole batch through csa_legacy_sample and return integer results.  ``devices``
    (a list of HIP device ids, repeats allowed) shards the panels over those devices of this
    process through csa_legacy_sample_devices; the results are identical."""
    S = int(iterations)
    flags = N.CSA_WANT_COUNTS | N.CSA_WANT_UNIQUE
    counts = np.zeros(enc.n, np.int64)
    pairs = np.zeros((enc.n, enc.n), np.int64) if want_pairs else None
    panels = np.zeros((S, enc.W), np.uint64) if want_panels else None
    attempts = np.zeros(S, np.uint32) if want_attempts else None
    unique = np.zeros(1, np.uint64)
    if want_pairs:
        flags |= N.CSA_WANT_PAIRS
    if want_panels:
        flags |= N.CSA_WANT_PANELS
    seed64 = int(random_seed) & 0xFFFFFFFFFFFFFFFF
    outs = (N.ptr(panels), N.ptr(counts), N.ptr(pairs), N.ptr(unique), N.ptr(attempts))
    reset_draw_stats(enc)
    if devices is None:
        rc = N.lib().csa_legacy_sample(enc.handle, int(k), seed64, panel_begin, S, flags, max_attempts, *outs)
    else:
        dev = np.ascontiguousarray(devices, np.int32)
        rc = N.lib().csa_legacy_sample_devices(enc.handle, N.ptr(dev), len(dev), int(k), seed64, panel_begin, S,
                                               flags, max_attempts, *outs)
    if rc == N.CSA_E_BAD_QUOTAS:
        raise AssertionError(N.last_error())     # analysis.py:174-176
    if rc == N.CSA_E_NO_CANDIDATE:
        raise KeyError("")                       # legacy.py:188
    N.check(rc)
    return LegacyRaw(counts, pairs, int(unique[0]), panels, attempts, draw_stats(enc))


def cached_pipeline(enc, k, chunk):
    """The encoding's DevicePipeline for draws of at most ``chunk`` panels per launch on the current
    device (picks / XT / pair scratch sized to one chunk, reused across calls; no n*n pair matrix of
    its own -- callers pass a fresh one per call).  Rebuilt when k, the device or a larger chunk
    asks for it."""
    import torch
    from .device import DevicePipeline
    pipe = getattr(enc, "_pipe", None)
    dev = torch.device("cuda", torch.cuda.current_device())
    if pipe is None or pipe.max_panels < int(chunk) or pipe.k != int(k) or pipe.device != dev:
        enc._pipe = None                      # release the old buffers before allocating new ones
        pipe = enc._pipe = DevicePipeline(enc, k, int(chunk), want_pairs=True, want_unique=True, pairs_buffer=False,
                                          device=dev)
    return pipe


def legacy_sample_device(enc, k, S, random_seed, keep_panels=True, chunk=1 << 20, host_panels=None,
                         host_stats=None):
    """One legacy_probabilities batch on the device through a DevicePipeline cached with the
    encoding (picks / XT / scratch buffers reused across calls).  Panels and hashes of the whole
    batch go to fresh device tensors (the exact distinct count needs all of them; with
    ``keep_panels`` the returned PanelSet keeps the panel tensor and decodes it only when
    iterated).  Returns LegacyRaw with host counts and device pair counts (PairHistogram
    materialises them lazily).  ``host_panels`` (uint64[S, W], MT mode: drawn on the host)
    replaces the device draw; the counting, pairs and distinct count still run on the device
    (``host_stats``: that draw's statistics)."""
    import torch
    from .distributed import HashTable
    S = int(S)
    C = max(1, min(S, int(chunk)))
    pipe = cached_pipeline(enc, k, C)
    W = enc.W
    dev = pipe.device
    with torch.cuda.device(dev), torch.cuda.stream(pipe.stream):
        panels = torch.empty(max(S * W, 1), dtype=torch.int64, device=dev)
        hashes = torch.empty(max(2 * S, 2), dtype=torch.int64, device=dev)
        pairs = torch.empty(enc.n * enc.n, dtype=torch.int64, device=dev)
        # status before the draws; the counters after the draws are enqueued (the draw stream does not
        # wait for them, the counting on this stream does).  A one-chunk call folds the status and
        # statistics resets into its draw call (csa_draw_xt_async).
        one = host_panels is None and 0 < S <= C and os.environ.get("CSA_DRAW_XT", "1") != "0"
        pipe.reset(pairs=False, counts=host_panels is not None, status=not one)
        if host_panels is None and not one:
            reset_draw_stats(enc, pipe.stream)
        own_p, own_h, own_pairs = pipe.panels, pipe.hashes, pipe.pairs
        pipe.pairs = pairs
        # the distinct-count table (zero-filled on allocation, on this stream) before the draws: the
        # draw stream waits on this stream, and the distinct count's side stream on the draw stream
        table = getattr(enc, "_table", None)
        if table is None or table.device != dev:
            table = enc._table = HashTable(S, dev)
        table.ensure(S)
        try:
            drawn = None  # what the distinct count's side stream waits for: the draws
            if one:
                # one chunk: draw on the pipeline stream; draw_lane_kernel's fused pack also writes the XT
                # blocks (csa_draw_xt_async), so the counting is the pair kernel alone and the counts
                # are the pair diagonal -- the transpose pass leaves the call's serial tail
                pipe.panels, pipe.hashes = panels[:S * W], hashes[:2 * S]
                xt_done = pipe.draw_xt(random_seed, 0, S, reset=True)
                drawn = torch.cuda.Event()
                drawn.record(pipe.stream)
                if not xt_done:
                    pipe.counts.zero_()
                    pipe.transpose_count(S)
                pipe.pair_counts(S, overwrite=True, alone=True)
                if xt_done:
                    pipe.counts_from_pairs()
            elif host_panels is None:
                # chunk draws on the pipeline's draw stream, counting and pairs on its stream, overlapped
                # (DevicePipeline.draw_count_chunks); two draw streams were measured slower
                # (profiles/r04f_draw_streams/)
                pipe.draw_count_chunks(random_seed, 0, S, panels, hashes, C, overwrite_pairs=True, reset_counts=True)
            else:
                for off in range(0, S, C):
                    ln = min(C, S - off)
                    pipe.panels, pipe.hashes = panels[off * W:(off + ln) * W], hashes[2 * off:2 * (off + ln)]
                    src = np.ascontiguousarray(host_panels[off:off + ln], np.uint64).view(np.int64).reshape(-1)
                    pipe.panels.copy_(torch.from_numpy(src), non_blocking=False)
                    pipe.hash(ln)
                    pipe.transpose_count(ln)
                    pipe.pair_counts(ln, overwrite=off == 0)
            if S == 0:
                pairs.zero_()
            # the distinct count needs only the draws (hashes, panels): with device draws it runs on a
            # side stream beside the counting and pairs of the last chunk, and the pipeline stream
            # waits for it before the one host read.  Everything it touches is ordered on that stream:
            # the counter reset, the table, and the hand-back (pipeline stream waits on the side stream)
            ust = pipe.stream
            if host_panels is None:
                ust = getattr(pipe, "unique_stream", None)
                if ust is None:
                    ust = pipe.unique_stream = torch.cuda.Stream(dev)
                if drawn is not None:
                    ust.wait_event(drawn)
                else:
                    ust.wait_stream(pipe.draw_stream)  # (the draw stream itself waited on the pipeline stream)
            with torch.cuda.stream(ust):
                table.count.zero_()
                N.check(N.lib().csa_unique_async(N.ptr(hashes), N.ptr(panels), S, W, N.ptr(table.table), table.slots,
                                                 N.ptr(table.count), N.ptr(pipe.status),
                                                 ctypes.c_void_p(ust.cuda_stream)))
            if ust is not pipe.stream:
                pipe.stream.wait_stream(ust)
            # counts, distinct count, draw statistics and status in ONE copy: the call's one host wait
            parts = [pipe.counts, table.count]
            if host_panels is None:
                st_d = torch.zeros(3, dtype=torch.int64, device=dev)
                N.check(N.lib().csa_instance_draw_stats_async(enc.handle, N.ptr(st_d),
                                                              ctypes.c_void_p(pipe.stream.cuda_stream)))
                parts.append(st_d)
            h = torch.cat(parts + [pipe.status.to(torch.int64)]).cpu().numpy()
            n_ = enc.n
            status = (h[-4:] & 0xFFFFFFFF).astype(np.uint32)
            if status[0]:
                rc = N.lib().csa_status_decode(N.ptr(status))
                if rc == N.CSA_E_NO_CANDIDATE:
                    raise KeyError("")       # legacy.py:188
                N.check(rc)
            counts = h[:n_].copy()
            unique = int(h[n_])
            stats = dict(zip(STAT_KEYS, (int(x) for x in h[n_ + 1:n_ + 4]))) if host_panels is None else host_stats
        finally:
            pipe.panels, pipe.hashes, pipe.pairs = own_p, own_h, own_pairs
    return LegacyRaw(counts, pairs.view(enc.n, enc.n), unique, panels[: S * W] if keep_panels else None, None,
                     stats)


def legacy_probabilities(instance: Instance, iterations: int, random_seed: int,
                         keep_panels: bool = True, rng: str = None,
                         devices=None) -> Tuple[ProbAllocation, PanelSet, PairHistogram]:
    """analysis.py:162-191 on the GPU.

    Returns ``({agent_id: count/S}, found_panels, pair_histogram)`` with the
    pair histogram divided by S, as the reference.  With torch.distributed
    initialised and world size > 1 the panels are sharded over ranks (see
    ``distributed.legacy_probabilities_distributed``).

    ``rng="mt"`` (default: ``legacy.RNG_MODE``) reproduces the reference's own
    stream: ``random.seed(random_seed)`` (analysis.py:169), then the panels are
    drawn on the host from the stdlib MT19937 state exactly as legacy.py:149
    consumes it (csa_legacy_draw_mt) and counted / paired / deduplicated on the
    device.  It matches the published reference_output probabilities.

    ``devices`` (Philox mode, one process): shard the panels over these HIP
    devices through csa_legacy_sample_devices instead of torch.distributed.

    A sharded run's found_panels hold no panels: reading them on any rank re-draws the job's panels
    on that rank's GPU (``distributed.PanelRedraw``), without a collective.
    """
    from . import distributed as D
    mode = rng or _legacy.RNG_MODE
    if mode not in ("philox", "mt"):
        raise ValueError("rng must be 'philox' or 'mt'")
    enc = encode_cached(instance.categories, instance.agents)
    S = int(iterations)
    if mode == "mt":
        import random
        random.seed(random_seed)
        np.random.seed(random_seed)                  # analysis.py:170 (unused by LEGACY)
        enc.check_quotas(instance.k)
        st = np.zeros(3, np.uint64)
        picks, panels, _ = mt_draw(enc, instance.k, S, stats=st)
        raw = legacy_sample_device(enc, instance.k, S, random_seed, keep_panels=keep_panels, host_panels=panels,
                                   host_stats=dict(zip(STAT_KEYS, (int(x) for x in st))))
        return finish(instance, enc, raw, S)
    if D.world_size() > 1:
        return D.legacy_probabilities_distributed(instance, iterations, random_seed, keep_panels=keep_panels)
    seed(random_seed)
    enc.check_quotas(instance.k)
    STREAM.take_panels(S)
    if devices is not None:
        raw = legacy_sample_raw(enc, instance.k, S, random_seed, want_pairs=True, want_panels=keep_panels,
                                devices=devices)
        return finish(instance, enc, raw, S)
    raw = legacy_sample_device(enc, instance.k, S, random_seed, keep_panels=keep_panels)
    return finish(instance, enc, raw, S)


def finish(instance, enc, raw, S):
    global LAST_RUN_STATS
    LAST_RUN_STATS = raw.stats
    # count / S as the reference's int / int true division: both operands are exact in float64 (< 2^53)
    # and IEEE division is correctly rounded, so numpy's float64 quotient is that same value
    alloc = dict(zip(enc.agent_ids, (np.asarray(raw.counts, dtype=np.float64) / float(S)).tolist())) if S else \
        {aid: int(c) / S for aid, c in zip(enc.agent_ids, np.asarray(raw.counts).tolist())}
    hist = PairHistogram(len(instance.agents), counts=raw.pairs)
    hist.turn_into_probabilities_by_dividing_all_elements_by_given_number(S)
    hist._counts, hist._S = raw.pairs, S      # integer counts for stats.sorted_pair_probabilities
    panels = PanelSet(raw.unique, raw.panels, enc.n, enc.agent_ids)
    return alloc, panels, hist
