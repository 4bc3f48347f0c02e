"""LEGACY result cache: run_legacy_or_retrieve.

The reference (analysis.py:271-293) pickles ``(alloc, found_panels, pair_histogram)``
to ``distributions/{name}_{k}_legacy_{first|second}.pickle`` (seed 0 / 1,
10,000 panels) and loads it on later runs.  A dict of n(n-1)/2 pair entries is
impractical at n = 8192 (33.5 M entries), so the cache here is a compact ``.npz``
of the exact integer results, written and read without pickle
(``numpy.load(allow_pickle=False)``):

    version, S, seed, k, n      scalars
    agent_ids                   int64[n] (or unicode[n]) in instance order
    counts                      int64[n] per-person counts
    pair_upper                  int32/int64[n(n-1)/2] pair counts, row-major i < j
                                (the reference's key order, analysis.py:70)
    unique                      distinct-panel count
    panels                      uint64[u, W] the distinct panels (optional)

Loading divides exactly as legacy_probabilities does (float64 true division), so a
retrieved result equals a fresh one bit for bit.  ``fmt="pickle"`` writes and reads
the reference's tuple shape with this package's classes; it is meant only for files
this module wrote.
"""
import os
import pickle
from pathlib import Path

import numpy as np

from .analysis import LegacyRaw, PairHistogram, PanelSet, finish, legacy_sample_raw
from .instance import encode
from .legacy import STREAM, seed as legacy_seed

CACHE_VERSION = 1


def legacy_cache_path(instance_name, k, resample, directory="distributions", fmt="npz"):
    """analysis.py:279-284 file naming ({name}_{k}_legacy_{first|second})."""
    stem = "%s_%d_legacy_%s" % (instance_name, int(k), "second" if resample else "first")
    return Path(directory, stem + (".pickle" if fmt == "pickle" else ".npz"))


def _ids_array(ids):
    if all(isinstance(a, (int, np.integer)) and not isinstance(a, bool) for a in ids):
        return np.asarray(ids, np.int64)
    return np.asarray([str(a) for a in ids])


def save_legacy_npz(path, enc, raw, S, random_seed, k, keep_panels=True):
    n = enc.n
    iu = np.triu_indices(n, 1)
    up = np.asarray(raw.pairs)[iu]
    if up.size and int(up.max()) < 2 ** 31:
        up = up.astype(np.int32)
    arrays = dict(version=np.int64(CACHE_VERSION), S=np.int64(S), seed=np.int64(random_seed), k=np.int64(k),
                  n=np.int64(n), agent_ids=_ids_array(enc.agent_ids), counts=np.asarray(raw.counts, np.int64),
                  pair_upper=up, unique=np.int64(raw.unique))
    if keep_panels and raw.panels is not None:
        arrays["panels"] = np.unique(np.ascontiguousarray(raw.panels, np.uint64), axis=0)
    tmp = str(path) + ".tmp.npz"
    np.savez_compressed(tmp, **arrays)
    os.replace(tmp, path)


def load_legacy_npz(path, instance):
    """-> (alloc, found_panels, pair_histogram), the reference's tuple (divided by S)."""
    with np.load(path, allow_pickle=False) as z:
        if int(z["version"]) != CACHE_VERSION:
            raise ValueError("%s: cache version %d, expected %d" % (path, int(z["version"]), CACHE_VERSION))
        enc = encode(instance.categories, instance.agents)
        n = int(z["n"])
        if n != enc.n or not np.array_equal(z["agent_ids"], _ids_array(enc.agent_ids)):
            raise ValueError("%s: cached agents do not match the instance" % path)
        S = int(z["S"])
        pairs = np.zeros((n, n), np.int64)
        pairs[np.triu_indices(n, 1)] = z["pair_upper"]
        np.fill_diagonal(pairs, z["counts"])   # X^T X diagonal = per-person counts, as a fresh result
        panels = z["panels"] if "panels" in z.files else None
        raw = LegacyRaw(z["counts"].astype(np.int64), pairs, int(z["unique"]), panels, None)
    return finish(instance, enc, raw, S)


def run_legacy_or_retrieve(instance_name, instance, resample, directory="distributions", fmt="npz",
                           iterations=10000, keep_panels=True):
    """analysis.py:271-293: load the cached LEGACY result or compute it (seed 0, or 1 when
    ``resample``) on the device and cache it."""
    path = legacy_cache_path(instance_name, instance.k, resample, directory, fmt)
    random_seed = 1 if resample else 0
    if path.exists():
        if fmt == "pickle":
            with open(path, "rb") as fh:            # only files this module wrote
                alloc, found_panels, pair_histogram = pickle.load(fh)
        else:
            alloc, found_panels, pair_histogram = load_legacy_npz(path, instance)
    else:
        legacy_seed(random_seed)
        enc = encode(instance.categories, instance.agents)
        enc.check_quotas(instance.k)
        S = int(iterations)
        STREAM.take_panels(S)
        raw = legacy_sample_raw(enc, instance.k, S, random_seed, want_pairs=True, want_panels=keep_panels)
        np.fill_diagonal(raw.pairs, raw.counts)
        alloc, found_panels, pair_histogram = finish(instance, enc, raw, S)
        Path(directory).mkdir(parents=True, exist_ok=True)
        if fmt == "pickle":
            with open(path, "wb") as fh:
                pickle.dump((alloc, found_panels, pair_histogram), fh)
        else:
            save_legacy_npz(path, enc, raw, S, random_seed, instance.k, keep_panels)
    assert len(alloc) == len(instance.agents)
    return alloc, found_panels, pair_histogram
