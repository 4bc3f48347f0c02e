"""Instances: the reference's dict form and its array encoding for the device.

``Instance`` / ``read_instance`` keep the reference's types and behaviour
(analysis.py:54-58, 108-138): ``categories[cat][feat] = {"min", "max",
"selected": 0, "remaining": pool count}`` in CSV order and ``agents[i] =
{cat: feat}`` with ``i`` the 0-based respondent row.

``encode`` turns any (categories, agents) dict pair into the arrays the C ABI
takes (include/csa_legacy.h): features numbered category-major in dict order
(the order find_max_ratio_cat scans them, legacy.py:129-130), agents numbered
in dict insertion order (the order the holder scan walks them,
legacy.py:187), so bit positions and ids map back one-to-one.
"""
import csv
from dataclasses import dataclass
from pathlib import Path
from typing import Any, Dict, Union

import numpy as np

from . import _native as N

AgentId = Any


@dataclass
class Instance:
    """analysis.py:54-58."""
    k: int
    categories: Dict[str, Dict[str, Dict[str, int]]]
    agents: Dict[AgentId, Dict[str, str]]


def read_instance(feature_file: Union[str, Path], pool_file: Union[str, Path], k: int) -> Instance:
    """analysis.py:108-138: categories in CSV order, agent id = row index."""
    feature_info = {}
    with open(feature_file, "r", encoding="utf-8") as fh:
        for line in csv.DictReader(fh):
            feature_info.setdefault(line["category"], {})[line["feature"]] = {
                "min": int(line["min"]), "max": int(line["max"]), "selected": 0, "remaining": 0}
    cats = list(feature_info)
    agents = {}
    with open(pool_file, "r", encoding="utf-8") as fh:
        for i, line in enumerate(csv.DictReader(fh)):
            agents[i] = {c: line[c] for c in cats}
            for c in cats:
                feature_info[c][line[c]]["remaining"] += 1   # KeyError on unknown feature, as the reference
    return Instance(k=k, categories=feature_info, agents=agents)


class EncodedInstance:
    """Array form of (categories, agents) plus the device-resident native handle."""

    def __init__(self, categories, agents):
        self.cat_names = list(categories)
        self.feat_keys = []                  # (category, feature) per global feature id
        fid = {}
        fmin, fmax, fcat, sel, rem = [], [], [], [], []
        for c, cat in enumerate(self.cat_names):
            for feat, info in categories[cat].items():
                fid[(cat, feat)] = len(self.feat_keys)
                self.feat_keys.append((cat, feat))
                fmin.append(int(info["min"]))
                fmax.append(int(info["max"]))
                fcat.append(c)
                sel.append(int(info.get("selected", 0)))
                rem.append(int(info["remaining"]) if "remaining" in info else -1)   # -1: the pool count
        self.agent_ids = list(agents)
        self.n = len(self.agent_ids)
        self.C = len(self.cat_names)
        self.F = len(self.feat_keys)
        self.W = (self.n + 63) // 64
        pf = np.empty((self.n, self.C), np.int32)
        for p, aid in enumerate(self.agent_ids):
            person = agents[aid]
            for c, cat in enumerate(self.cat_names):
                pf[p, c] = fid[(cat, person[cat])]
        self.person_feat = pf
        self.fmin = np.asarray(fmin, np.int32)
        self.fmax = np.asarray(fmax, np.int32)
        self.fcat = np.asarray(fcat, np.int32)
        self.sel0 = np.asarray(sel, np.int32)
        self.rem0 = np.asarray(rem, np.int32)
        self.pool = np.bincount(pf.ravel(), minlength=self.F).astype(np.int32) if self.n else \
            np.zeros(self.F, np.int32)
        self.rem0 = np.where(self.rem0 < 0, self.pool, self.rem0).astype(np.int32)
        self._handles = {}                   # HIP device index -> native instance on that device

    # -- native handle ---------------------------------------------------------------------
    @property
    def handle(self):
        """The native instance on the calling thread's current HIP device (created there on first use).
        The stream-ordered entry points launch on the caller's stream, so an instance must live on the
        device the call runs on: a sharded call runs on its rank's GPU without changing the caller's
        current device, and a later call on another device gets an instance of its own."""
        import ctypes
        L = N.lib()
        d = ctypes.c_int32(-1)
        N.check(L.csa_current_device(ctypes.byref(d)))
        h = self._handles.get(d.value)
        if h is None:
            h = ctypes.c_void_p()
            N.check(L.csa_instance_create(self.n, self.C, self.F, N.ptr(self.person_feat), N.ptr(self.fmin),
                                          N.ptr(self.fmax), N.ptr(self.fcat), ctypes.byref(h)))
            self._handles[d.value] = h
            # the dicts' own "selected" / "remaining" counters are the draw's start state, as in
            # the reference's deep copies (analysis.py:147-148); the device default is 0 / pool
            if np.any(self.sel0 != 0) or not np.array_equal(self.rem0, self.pool):
                N.check(L.csa_instance_set_state(h, N.ptr(self.sel0), N.ptr(self.rem0), None))
        return h

    def release_device_buffers(self):
        """Drop the cached device pipeline / hash table (they are rebuilt on the next call)."""
        self.__dict__.pop("_pipe", None)
        self.__dict__.pop("_table", None)

    def close(self):
        handles, self._handles = getattr(self, "_handles", {}), {}
        for h in handles.values():
            N.lib().csa_instance_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check_quotas(self, k):
        """analysis.py:174-176 (AssertionError, as the reference).  A passing k is remembered (the
        encoding's quotas never change)."""
        ok = self.__dict__.setdefault("_quota_ok", set())
        if k in ok:
            return
        for c in range(self.C):
            m = self.fcat == c
            assert int(self.fmin[m].sum()) <= k
            assert int(self.fmax[m].sum()) >= k
        ok.add(k)

    # -- helpers ---------------------------------------------------------------------------
    def present_mask(self, keys=None):
        """uint64[W] bitmask of the agents in ``keys`` (default: all)."""
        out = np.zeros(self.W, np.uint64)
        pos = range(self.n) if keys is None else [self.agent_ids.index(a) for a in keys]
        for p in pos:
            out[p >> 6] |= np.uint64(1) << np.uint64(p & 63)
        return out


def encode(categories, agents) -> EncodedInstance:
    return EncodedInstance(categories, agents)


_ENC_CACHE = []        # [(categories, agents, fingerprint, EncodedInstance)], most recent last
_ENC_CACHE_SIZE = 4


def _fingerprint(categories, agents):
    return (tuple((c, f, v["min"], v["max"], v.get("selected", 0), v.get("remaining", 0))
                  for c in categories for f, v in categories[c].items()), tuple(agents))


def encode_cached(categories, agents) -> EncodedInstance:
    """``encode`` memoised for callers that draw repeatedly from the same dicts (XMIN's
    3n-fold legacy_find loop, xmin.py:464-474, called 5n times): the entry is keyed by the
    dict objects themselves (held, so their ids stay unique) and revalidated by the feature
    quotas / counters and the agent ids.  In-place edits of a person's feature values are
    not detected -- the reference's callers never make them."""
    fp = _fingerprint(categories, agents)
    for i, (c, a, f, enc) in enumerate(_ENC_CACHE):
        if c is categories and a is agents and f == fp:
            _ENC_CACHE.append(_ENC_CACHE.pop(i))
            return enc
    enc = EncodedInstance(categories, agents)
    _ENC_CACHE.append((categories, agents, fp, enc))
    for entry in _ENC_CACHE[:-_ENC_CACHE_SIZE]:
        # an evicted entry's device buffers (analysis.legacy_sample_device's pipeline and
        # distinct-count table) go now, not when the last reference to the encoding goes
        entry[3].release_device_buffers()
    del _ENC_CACHE[:-_ENC_CACHE_SIZE]
    return enc


def unpack_panel(words, n):
    """uint64[W] -> sorted list of bit positions."""
    bits = np.unpackbits(np.ascontiguousarray(words, np.uint64).view(np.uint8), bitorder="little")[:n]
    return np.flatnonzero(bits).tolist()
