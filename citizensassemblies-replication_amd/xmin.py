"""XMIN's LEGACY caller on the device.

``_get_panel_not_in_portfolio_if_possible`` (xmin.py:464-474) calls ``legacy_find``
up to 3n times and returns the first panel (a frozenset of agent ids) that is not
in the portfolio, or None.  Here the candidate panels are drawn in growing chunks
by the draw kernel and tested against a device hash table of the portfolio
(``csa_first_panel_not_in``); the Philox stream advances by exactly the number of
``legacy_find`` calls the reference makes (index of the first non-member + 1, or
3n), so later draws are unchanged.  The rest of XMIN (Gurobi column generation)
stays on the CPU, outside this package.
"""
import ctypes

import numpy as np

from . import _native as N
from . import legacy as _legacy
from .instance import encode_cached, unpack_panel
from .legacy import STREAM, mt_draw


_ROW_CACHE = {}      # id(enc) -> (enc, {panel: packed row or None}); XMIN's portfolio grows by one per call
_MISSING = object()


def _pack_one(pos, W, panel):
    row = np.zeros(W, np.uint64)
    for aid in panel:
        p = pos.get(aid)
        if p is None:
            return None
        row[p >> 6] |= np.uint64(1) << np.uint64(p & 63)
    return row


def pack_portfolio(enc, portfolio):
    """Portfolio panels (iterables of agent ids) -> uint64[m, W] packed bitmasks.

    Panels naming an agent outside the instance can never equal a drawn panel and
    are left out (membership of drawn panels is unchanged).  Rows of hashable panels
    (frozensets, as XMIN's portfolio holds) are memoised per encoding."""
    ent = _ROW_CACHE.get(id(enc))
    if ent is None or ent[0] is not enc:
        _ROW_CACHE.clear()
        ent = _ROW_CACHE[id(enc)] = (enc, {}, {aid: p for p, aid in enumerate(enc.agent_ids)})
    _, memo, pos = ent
    rows = []
    for panel in portfolio:
        if isinstance(panel, frozenset):
            row = memo.get(panel, _MISSING)
            if row is _MISSING:
                row = memo[panel] = _pack_one(pos, enc.W, panel)
        else:
            row = _pack_one(pos, enc.W, panel)
        if row is not None:
            rows.append(row)
    if not rows:
        return np.zeros((0, enc.W), np.uint64)
    return np.ascontiguousarray(np.stack(rows))


def first_panel_not_in(enc, k, seed, panel_begin, n_panels, packed_portfolio, chunk=256, max_attempts=0):
    """Offset of the first panel in [panel_begin, panel_begin + n_panels) that is not in the
    packed portfolio, and that panel's bitmask; (-1, None) if every one is a member."""
    idx = ctypes.c_int64(-1)
    panel = np.zeros(max(enc.W, 1), np.uint64)
    port = np.ascontiguousarray(packed_portfolio, np.uint64)
    N.check(N.lib().csa_first_panel_not_in(enc.handle, int(k), int(seed) & 0xFFFFFFFFFFFFFFFF, int(panel_begin),
                                           int(n_panels), int(max_attempts), N.ptr(port) if len(port) else None,
                                           len(port), int(chunk), ctypes.byref(idx), N.ptr(panel)))
    return (idx.value, panel) if idx.value >= 0 else (-1, None)


def _get_panel_not_in_portfolio_if_possible(categories, agents, k, portfolio, chunk=256, rng=None):
    """xmin.py:464-474 (same arguments, result and stream consumption).  In MT mode (rng="mt" /
    legacy.RNG_MODE) the legacy_find calls draw one by one from the stdlib random stream, as the
    reference does, and the membership test stays on the host."""
    enc = encode_cached(categories, agents)
    tries = len(agents) * 3
    if (rng or _legacy.RNG_MODE) == "mt":
        members = {frozenset(p) for p in portfolio}
        for _ in range(tries):
            picks, _, _ = mt_draw(enc, k, 1)
            panel = frozenset(enc.agent_ids[int(p)] for p in picks[0] if p >= 0)
            if panel not in members:
                return panel
        return None
    first = STREAM.panel
    j, words = first_panel_not_in(enc, k, STREAM.key, first, tries, pack_portfolio(enc, portfolio), chunk=chunk)
    STREAM.take_panels(j + 1 if j >= 0 else tries)
    if j < 0:
        return None
    return frozenset(enc.agent_ids[p] for p in unpack_panel(words, enc.n))
