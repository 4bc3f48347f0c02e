"""Pure-Python restatement of the reference LEGACY Monte Carlo path.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): used by tests/ as the
checker, never by the product.

What it restates (reference file:line):
  * read_instance            analysis.py:108-138  (CSV order = feature order,
                                                   agent id = 0-based row index)
  * find_max_ratio_cat       legacy.py:124-157    (a5: FAIL test, candidate test,
                                                   strict '>' argmax from -100.0,
                                                   randint on every improvement)
  * holder scan              legacy.py:186-197    (a6: r-th remaining holder in
                                                   ascending agent id)
  * delete_person            legacy.py:103-120, 67-75 (a7)
  * delete_all_in_cat        legacy.py:47-62      (a8, bulk order-free form)
  * find_random_sample_legacy legacy.py:178-200   (k steps + empty-pool test)
  * check_min_cats           legacy.py:160-168    (a9)
  * legacy_find              analysis.py:141-159  (restart on SelectionError,
                                                   retry on min-quota rejection)
  * legacy_probabilities     analysis.py:162-191  (counts, pair histogram,
                                                   distinct panels)

The ratio comparison ``(min-sel)/float(rem) > best`` (legacy.py:141-145) is
restated as exact integer cross-multiplication; that is equivalent because the
ratios are quotients of small integers (|num| <= k, 1 <= den <= n < 2**26),
for which float64 division is injective and monotone.

RNG modes
  * ``"mt"``:     stdlib ``random.Random(seed).randint(1, rem)`` called at every
                  improvement, exactly the reference call pattern
                  (legacy.py:149, seeded at analysis.py:169).  Pinned by the
                  reference's published CSVs.
  * ``"philox"``: the verification-mode stream of oracle/philox.py (the stream
                  the GPU kernel implements), keyed by (seed, panel, attempt, step).
"""
import csv
import random
from dataclasses import dataclass, field

import numpy as np

from .philox import legacy_word, legacy_randint

OK, FAIL, REJECT = 0, 1, 2


class NoCandidateError(KeyError):
    """Mirrors the reference's KeyError at legacy.py:188 (no candidate feature)."""


@dataclass
class OracleInstance:
    k: int
    cat_names: list            # category names, CSV order
    feat_names: list           # (category, feature) per global feature index
    fmin: list
    fmax: list
    fcat: list                 # category index of each feature
    person_feat: list          # person_feat[p][c] = global feature index
    agent_ids: list = field(default_factory=list)

    @property
    def n(self):
        return len(self.person_feat)

    @property
    def F(self):
        return len(self.fmin)

    @property
    def C(self):
        return len(self.cat_names)

    def pool_counts(self):
        rem = [0] * self.F
        for feats in self.person_feat:
            for g in feats:
                rem[g] += 1
        return rem


def read_instance(cat_csv, resp_csv, k):
    """Restates analysis.py:108-138 into arrays (feature order = CSV row order)."""
    cat_names, feat_names, fmin, fmax, fcat = [], [], [], [], []
    index = {}
    with open(cat_csv, "r", encoding="utf-8") as fh:
        for row in csv.DictReader(fh):
            c, f = row["category"], row["feature"]
            if c not in cat_names:
                cat_names.append(c)
            key = (c, f)
            if key in index:          # dict assignment in the reference overwrites
                g = index[key]
                fmin[g], fmax[g] = int(row["min"]), int(row["max"])
                continue
            index[key] = len(feat_names)
            feat_names.append(key)
            fmin.append(int(row["min"]))
            fmax.append(int(row["max"]))
            fcat.append(cat_names.index(c))
    # the reference groups features by category (nested dict), so global order is
    # category-major in first-appearance order of the category
    order = sorted(range(len(feat_names)), key=lambda g: (fcat[g], g))
    remap = {old: new for new, old in enumerate(order)}
    feat_names = [feat_names[g] for g in order]
    fmin = [fmin[g] for g in order]
    fmax = [fmax[g] for g in order]
    fcat = [fcat[g] for g in order]
    index = {key: remap[g] for key, g in index.items()}
    person_feat = []
    with open(resp_csv, "r", encoding="utf-8") as fh:
        for row in csv.DictReader(fh):
            person_feat.append([index[(c, row[c])] for c in cat_names])
    return OracleInstance(k=k, cat_names=cat_names, feat_names=feat_names, fmin=fmin,
                          fmax=fmax, fcat=fcat, person_feat=person_feat,
                          agent_ids=list(range(len(person_feat))))


def draw_attempt(inst, k, rng, sel=None, rem=None, present=None):
    """One call of find_random_sample_legacy (legacy.py:178-200) on array state.

    ``rng(step, rem_f)`` is invoked at every argmax improvement (legacy.py:149).
    Returns (status, picks, sel, rem, present); status OK or FAIL (SelectionError).
    Raises NoCandidateError where the reference raises KeyError (legacy.py:188).
    """
    F, n = inst.F, inst.n
    fmin, fmax, fcat, pf = inst.fmin, inst.fmax, inst.fcat, inst.person_feat
    sel = list(sel) if sel is not None else [0] * F
    rem = list(rem) if rem is not None else inst.pool_counts()
    present = list(present) if present is not None else [True] * n
    picks = []
    for step in range(k):
        # a5: find_max_ratio_cat (legacy.py:124-157)
        best = None
        r = -1
        for f in range(F):
            need = fmin[f] - sel[f]
            if sel[f] < fmin[f] and rem[f] < need:
                return FAIL, picks, sel, rem, present
            if rem[f] != 0 and fmax[f] != 0:
                if best is None:
                    better = need > -100 * rem[f]          # ratio > -100.0
                else:
                    better = need * best[1] > best[0] * rem[f]
                if better:
                    best = (need, rem[f], f)
                    r = rng(step, rem[f])
        any_present = any(present)
        if best is None:
            if any_present:
                raise NoCandidateError("no candidate feature at step %d" % step)
        else:
            # a6: r-th remaining holder of f* in ascending agent order
            fs = best[2]
            c = fcat[fs]
            pick = None
            for p in range(n):
                if present[p] and pf[p][c] == fs:
                    r -= 1
                    if r == 0:
                        pick = p
                        break
            if pick is not None:
                picks.append(pick)
                # a7: really_delete_person(selected=True)
                present[pick] = False
                for g in pf[pick]:
                    sel[g] += 1
                    rem[g] -= 1
                # a8: cascade for the picked person's full features (bulk form)
                full = [g for g in pf[pick] if sel[g] == fmax[g]]
                if full:
                    for q in range(n):
                        if present[q] and any(pf[q][fcat[g]] == g for g in full):
                            present[q] = False
                            for g in pf[q]:
                                rem[g] -= 1
                for g in range(F):
                    if rem[g] == 0 and sel[g] < fmin[g]:
                        return FAIL, picks, sel, rem, present
        # legacy.py:198-199
        if step < k - 1 and not any(present):
            return FAIL, picks, sel, rem, present
    return OK, picks, sel, rem, present


def check_min_cats(inst, sel):
    """legacy.py:160-168."""
    return all(sel[f] >= inst.fmin[f] for f in range(inst.F))


class PhiloxRng:
    """Verification-mode stream: per (seed, panel, attempt) a fresh rng(step, rem)."""

    def __init__(self, seed):
        self.seed = seed

    def for_attempt(self, panel, attempt):
        seed = self.seed

        def rng(step, rem_f):
            return legacy_randint(legacy_word(seed, panel, attempt, step), rem_f)
        return rng


class MtRng:
    """stdlib MT19937 exactly as the reference consumes it (one shared stream)."""

    def __init__(self, seed):
        self.r = random.Random(seed)

    def for_attempt(self, panel, attempt):
        r = self.r

        def rng(step, rem_f):
            return r.randint(1, rem_f)
        return rng


def legacy_find(inst, k, rng_src, panel, max_attempts=1 << 20):
    """analysis.py:141-159.  Returns (picks in pick order, attempts used)."""
    attempt = 0
    while attempt < max_attempts:
        status, picks, sel, _rem, _present = draw_attempt(inst, k, rng_src.for_attempt(panel, attempt))
        attempt += 1
        if status == FAIL:
            continue
        if check_min_cats(inst, sel):
            return picks, attempt
    raise RuntimeError("attempt limit reached for panel %d" % panel)


@dataclass
class OracleResult:
    counts: np.ndarray          # int64[n]
    pairs: np.ndarray           # int64[n,n], upper triangle i<j valid, diag = counts
    panels: list                # sorted tuples, panel order
    picks: list                 # pick order lists
    attempts: list              # attempts used per panel (>=1)

    @property
    def unique(self):
        return len(set(self.panels))


def legacy_probabilities(inst, S, seed, mode="philox", panel_begin=0, want_pairs=True):
    """analysis.py:162-191 restated; returns raw integer results."""
    for c in range(inst.C):                       # analysis.py:174-176
        feats = [g for g in range(inst.F) if inst.fcat[g] == c]
        assert sum(inst.fmin[g] for g in feats) <= inst.k
        assert sum(inst.fmax[g] for g in feats) >= inst.k
    src = PhiloxRng(seed) if mode == "philox" else MtRng(seed)
    n = inst.n
    counts = np.zeros(n, np.int64)
    panels, picks_all, attempts = [], [], []
    X = np.zeros((S, n), np.float64) if want_pairs else None
    for i in range(S):
        picks, att = legacy_find(inst, inst.k, src, panel_begin + i)
        panel = tuple(sorted(picks))
        panels.append(panel)
        picks_all.append(picks)
        attempts.append(att)
        counts[list(panel)] += 1
        if want_pairs:
            X[i, list(panel)] = 1.0
    if want_pairs:
        pairs = np.rint(X.T @ X).astype(np.int64)   # exact: entries <= S < 2**53
    else:
        pairs = None
    return OracleResult(counts=counts, pairs=pairs, panels=panels, picks=picks_all, attempts=attempts)


def pack_panels(panels, n):
    """Sorted tuples -> uint64[S, ceil(n/64)] bitmasks (bit p%64 of word p//64)."""
    W = (n + 63) // 64
    out = np.zeros((len(panels), W), np.uint64)
    for i, panel in enumerate(panels):
        for p in panel:
            out[i, p >> 6] |= np.uint64(1) << np.uint64(p & 63)
    return out
