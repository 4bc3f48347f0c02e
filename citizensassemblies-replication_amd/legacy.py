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

# "philox": the device path (verification-mode stream above); "mt": the reference's own stdlib
# random stream, drawn on the host (csa_legacy_draw_mt) -- set_rng_mode switches the default
RNG_MODE = "philox"


def set_rng_mode(mode):
    global RNG_MODE
    if mode not in ("philox", "mt"):
        raise ValueError("rng mode must be 'philox' or 'mt'")
    RNG_MODE = mode


def seed(seed_value):
    """Counterpart of ``random.seed`` for the LEGACY draws (analysis.py:169)."""
    STREAM.seed(seed_value)


def mt_draw(enc, k, n_panels, single=False, max_attempts=0, state=False, addr_next=None, stats=None):
    """MT19937 mode: ``n_panels`` legacy_find calls (``single``: one find_random_sample_legacy
    call) drawing from the stdlib ``random`` module's global state exactly as legacy.py:149
    does; the state is advanced in place (random.setstate), also when the draw raises.
    Returns (picks int32[n_panels, k], panels uint64[n_panels, W], attempts) and, with
    ``state``, the final (sel, rem, present) of the single attempt.  ``stats`` (uint64[3], optional)
    receives the call's attempts, SelectionErrors and min-quota rejections."""
    import random
    k = int(k)
    st = random.getstate()
    words = np.array(st[1], dtype=np.uint32)
    picks = np.full((n_panels, max(k, 1)), -1, np.int32)
    panels = np.zeros((n_panels, max(enc.W, 1)), np.uint64)
    attempts = np.zeros(max(n_panels, 1), np.uint32)
    sel = np.zeros(enc.F, np.int32)
    rem = np.zeros(enc.F, np.int32)
    present = np.zeros(max(enc.W, 1), np.uint64)
    try:
        rc = N.lib().csa_legacy_draw_mt(enc.n, enc.C, enc.F, N.ptr(enc.person_feat), N.ptr(enc.fmin), N.ptr(enc.fmax),
                                        N.ptr(enc.sel0), N.ptr(enc.rem0), None, N.ptr(addr_next), k, N.ptr(words),
                                        int(n_panels),
                                        max_attempts, 1 if single else 0, N.ptr(picks), N.ptr(panels),
                                        N.ptr(attempts), N.ptr(sel), N.ptr(rem), N.ptr(present), N.ptr(stats))
    finally:
        random.setstate((st[0], tuple(int(x) for x in words), st[2]))
    if rc == N.CSA_E_SELECTION:
        raise SelectionError("FAIL: LEGACY attempt reached a dead end")
    if rc == N.CSA_E_NO_CANDIDATE:
        raise KeyError("")          # legacy.py:188
    N.check(rc)
    out = (picks[:, :k], panels[:, :enc.W], attempts[:n_panels])
    return out + ((sel, rem, present),) if state else out


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


def address_rings(agent_ids, columns_data, check_same_address_columns):
    """addr_next for csa_instance_set_address / csa_legacy_draw_mt: the agents whose
    (address1, zip) values in ``columns_data`` are equal -- get_people_at_same_address's test,
    legacy.py:81-92 -- linked into rings in agent order (a lone agent points to itself)."""
    c0, c1 = check_same_address_columns[0], check_same_address_columns[1]
    groups = {}
    for p, aid in enumerate(agent_ids):
        row = columns_data[aid]
        groups.setdefault((row[c0], row[c1]), []).append(p)
    nxt = np.arange(len(agent_ids), dtype=np.int32)
    for members in groups.values():
        for j, p in enumerate(members):
            nxt[p] = members[(j + 1) % len(members)]
    return nxt


def output_lines(categories, people, picks, columns_data, check_same_address, check_same_address_columns,
                 addr_next=None, agent_pos=None):
    """The reference's log lines of a successful attempt (legacy.py:95-97, 119, 182), rebuilt
    from the pick order: the deletions are a deterministic function of the picks.  Returns
    (lines, selected, remaining) counters after the attempt, (cat, feat) -> int."""
    lines = ["Using legacy algorithm."]
    sel = {(c, f): v["selected"] for c in categories for f, v in categories[c].items()}
    rem = {(c, f): v["remaining"] for c in categories for f, v in categories[c].items()}
    left = dict(people)
    ids = list(people) if agent_pos is not None else None
    for pkey in picks:
        person = left.pop(pkey)
        for c, f in person.items():
            sel[(c, f)] += 1
            rem[(c, f)] -= 1
        if check_same_address:
            a1 = columns_data[pkey][check_same_address_columns[0]]
            z = columns_data[pkey][check_same_address_columns[1]]
            p0 = agent_pos[pkey]
            q = int(addr_next[p0])
            while q != p0:
                qkey = ids[q]
                if qkey in left:
                    lines.append("Found someone with the same address as a selected person,"
                                 " so deleting him/her. Address: {} , {}".format(a1, z))
                    for c, f in left.pop(qkey).items():
                        rem[(c, f)] -= 1
                q = int(addr_next[q])
        for c, f in person.items():
            if sel[(c, f)] == categories[c][f]["max"]:
                gone = [q for q, pq in left.items() if pq[c] == f]
                for q in gone:
                    for c2, f2 in left.pop(q).items():
                        rem[(c2, f2)] -= 1
                lines.append("Category {} full - deleted {}, {} left.".format(f, len(gone), len(left)))
    return lines, sel, rem


def find_random_sample_legacy(categories: Dict[str, Dict[str, Dict[str, int]]], people: Dict[str, Dict[str, str]],
                              columns_data: Dict[str, Dict[str, str]], number_people_wanted: int,
                              check_same_address: bool, check_same_address_columns: List[str], *,
                              rng: str = None) -> Tuple[Dict[str, Dict[str, str]], List[str]]:
    """One LEGACY attempt (legacy.py:178-200): on the GPU (draw_kernel, Philox verification-mode
    stream) or, with rng="mt" (default: RNG_MODE), on the host from the stdlib random stream.

    On success the dicts are updated in place exactly as the reference leaves
    them (selected/remaining counters, picked, same-address and cascaded people
    removed from ``people``) and ``(people_selected, output_lines)`` is returned
    with ``people_selected`` in pick order and the reference's log lines.  On a
    dead end SelectionError is raised (the dicts are left untouched; the
    reference leaves them half-updated, and every caller discards them).  With
    ``check_same_address`` every pick also deletes the remaining people whose
    ``check_same_address_columns`` (address, zip) values equal the pick's
    (legacy.py:78-99, 109-113).
    """
    k = int(number_people_wanted)
    enc = encode(categories, people)
    ring = address_rings(enc.agent_ids, columns_data, check_same_address_columns) if check_same_address else None
    if (rng or RNG_MODE) == "mt":
        picks_a, _, _, (sel, rem, present) = mt_draw(enc, k, 1, single=True, state=True, addr_next=ring)
        picks = [int(p) for p in picks_a[0] if p >= 0]
    else:
        L = N.lib()
        h = enc.handle
        N.check(L.csa_instance_set_state(h, N.ptr(enc.sel0), N.ptr(enc.rem0), None))
        N.check(L.csa_instance_set_address(h, N.ptr(ring)))
        panel, attempt = STREAM.take_attempt()
        pk = np.full(max(k, 1), -1, np.int32)
        npk = ctypes.c_int32(0)
        sel = np.zeros(enc.F, np.int32)
        rem = np.zeros(enc.F, np.int32)
        present = np.zeros(max(enc.W, 1), np.uint64)
        rc = L.csa_legacy_attempt(h, k, STREAM.key, panel, attempt, N.ptr(pk), ctypes.byref(npk), N.ptr(sel),
                                  N.ptr(rem), N.ptr(present))
        if rc == N.CSA_E_SELECTION:
            raise SelectionError("FAIL: LEGACY attempt reached a dead end")
        if rc == N.CSA_E_NO_CANDIDATE:
            raise KeyError("")          # the reference looks up pvalue[""] (legacy.py:188)
        N.check(rc)
        picks = [int(p) for p in pk[:npk.value]]
    ids = enc.agent_ids
    pick_ids = [ids[p] for p in picks]
    lines, sel_r, rem_r = output_lines(categories, people, pick_ids, columns_data, check_same_address,
                                       check_same_address_columns, ring,
                                       {aid: p for p, aid in enumerate(ids)} if check_same_address else None)
    for g, (cat, feat) in enumerate(enc.feat_keys):
        if (sel_r[(cat, feat)], rem_r[(cat, feat)]) != (int(sel[g]), int(rem[g])):
            raise RuntimeError("device state disagrees with the replayed deletions at %s/%s" % (cat, feat))
        item = categories[cat][feat]
        item["selected"] = int(sel[g])
        item["remaining"] = int(rem[g])
    people_selected = {}
    for aid in pick_ids:
        people_selected[aid] = people[aid]
    for p, aid in enumerate(ids):
        if not (int(present[p >> 6]) >> (p & 63)) & 1:
            del people[aid]
    return people_selected, lines
