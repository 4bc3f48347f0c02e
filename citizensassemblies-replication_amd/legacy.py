"""Drop-in for the reference's legacy.py call surface, backed by the gfx950 draw kernel.

Kept names and semantics (reference file:line):
  * ``SelectionError``            legacy.py:34-36
  * ``check_min_cats``            legacy.py:160-168 (pure host logic, unchanged)
  * ``find_random_sample_legacy`` legacy.py:178-200 -- one attempt, mutates
    ``categories`` / ``people`` in place on success, raises SelectionError on a
    dead end and KeyError where the reference hits legacy.py:188.

Randomness: the reference draws from the global MT19937 stream
(``random.randint``, legacy.py:149).  Here every draw comes from the
Philox4x32-10 verification-mode stream keyed by (seed, panel, attempt, step)
-- see oracle/philox.py for the contract; ``seed()`` plays the role of
``random.seed`` (analysis.py:169).  The module-level stream advances like the
reference's hidden state: each ``legacy_find`` consumes one panel index, each
direct ``find_random_sample_legacy`` call consumes one attempt of the current
panel.
"""
import ctypes
from typing import Dict, List, Tuple

import numpy as np

from . import _native as N
from .instance import encode


class SelectionError(Exception):
    """legacy.py:34-36."""

    def __init__(self, message):
        super().__init__(message)
        self.msg = message


class LegacyStream:
    """Philox stream position: (seed, next panel index, next attempt of that panel)."""

    def __init__(self, seed_value=0):
        self.seed(seed_value)

    def seed(self, seed_value):
        self.key = int(seed_value) & 0xFFFFFFFFFFFFFFFF
        self.panel = 0
        self.attempt = 0

    def take_panels(self, count):
        first = self.panel
        self.panel += int(count)
        self.attempt = 0
        return first

    def take_attempt(self):
        a = self.attempt
        self.attempt += 1
        return self.panel, a


STREAM = LegacyStream(0)


def seed(seed_value):
    """Counterpart of ``random.seed`` for the LEGACY draws (analysis.py:169)."""
    STREAM.seed(seed_value)


def check_min_cats(categories):
    """legacy.py:160-168."""
    output_msg = []
    got_min = True
    for cats in categories.values():
        for cat, cat_item in cats.items():
            if cat_item["selected"] < cat_item["min"]:
                got_min = False
                output_msg = ["Failed to get minimum in category: {}".format(cat)]
    return got_min, output_msg


def find_random_sample_legacy(categories: Dict[str, Dict[str, Dict[str, int]]], people: Dict[str, Dict[str, str]],
                              columns_data: Dict[str, Dict[str, str]], number_people_wanted: int,
                              check_same_address: bool, check_same_address_columns: List[str]) \
        -> Tuple[Dict[str, Dict[str, str]], List[str]]:
    """One LEGACY attempt on the GPU (legacy.py:178-200).

    On success the dicts are updated in place exactly as the reference leaves
    them (selected/remaining counters, picked and cascaded people removed from
    ``people``) and ``(people_selected, output_lines)`` is returned with
    ``people_selected`` in pick order.  On a dead end SelectionError is raised
    (the dicts are left untouched; the reference leaves them half-updated, and
    every caller discards them).
    """
    if check_same_address:
        # legacy.py:78-99/109-113: never exercised by the LEGACY harness
        # (analysis.py:150-151 passes False); no device implementation.
        raise NotImplementedError("check_same_address=True is not supported by the GPU LEGACY path")
    k = int(number_people_wanted)
    enc = encode(categories, people)
    L = N.lib()
    h = enc.handle
    N.check(L.csa_instance_set_state(h, N.ptr(enc.sel0), N.ptr(enc.rem0), None))
    panel, attempt = STREAM.take_attempt()
    picks = np.full(max(k, 1), -1, np.int32)
    npk = ctypes.c_int32(0)
    sel = np.zeros(enc.F, np.int32)
    rem = np.zeros(enc.F, np.int32)
    present = np.zeros(max(enc.W, 1), np.uint64)
    rc = L.csa_legacy_attempt(h, k, STREAM.key, panel, attempt, N.ptr(picks), ctypes.byref(npk), N.ptr(sel),
                              N.ptr(rem), N.ptr(present))
    if rc == N.CSA_E_SELECTION:
        raise SelectionError("FAIL: LEGACY attempt reached a dead end")
    if rc == N.CSA_E_NO_CANDIDATE:
        raise KeyError("")          # the reference looks up pvalue[""] (legacy.py:188)
    N.check(rc)
    for g, (cat, feat) in enumerate(enc.feat_keys):
        item = categories[cat][feat]
        item["selected"] = int(sel[g])
        item["remaining"] = int(rem[g])
    people_selected = {}
    for p in picks[:npk.value]:
        aid = enc.agent_ids[int(p)]
        people_selected[aid] = people[aid]
    for p, aid in enumerate(enc.agent_ids):
        if not (int(present[p >> 6]) >> (p & 63)) & 1:
            del people[aid]
    return people_selected, ["Using legacy algorithm."]
