"""check_same_address on the GPU (legacy.py:78-99, 103-113),
Philox verification mode, against the reference's own runs (tests/golden/address_*.json,
"philox": tools/make_goldens.py drove the unmodified find_random_sample_legacy with
check_same_address=True in a legacy_find-shaped restart loop).

The same-address deletion runs in draw_kernel<64, ..., true> (csa_instance_set_address routes
every draw of the instance there): pick orders, attempt counts, per-person counts, single
attempts with their dict mutations and log lines must all be bit-exact.
"""
import copy
import csv
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLD, REPO, inst_paths, pkg

pytestmark = pytest.mark.gpu

ADDR = sorted(f[:-5] for f in os.listdir(GOLD) if f.startswith("address_") and f.endswith(".json"))


def _load(case):
    with open(os.path.join(GOLD, case + ".json")) as fh:
        g = json.load(fh)["philox"]
    with open(os.path.join(REPO, g["addresses"]), encoding="utf-8") as fh:
        cols = {i: dict(r) for i, r in enumerate(csv.DictReader(fh))}
    return g, cols


@pytest.mark.parametrize("case", ADDR)
def test_address_legacy_find_and_sample(gpu_available, case):
    g, cols = _load(case)
    P = pkg()
    L = pkg("legacy")
    N = pkg("_native")
    inst = P.read_instance(*inst_paths(g["instance"]), g["k"])
    enc = P.encode(inst.categories, inst.agents)
    ring = L.address_rings(enc.agent_ids, cols, g["columns"])
    lib = N.lib()
    N.check(lib.csa_instance_set_address(enc.handle, N.ptr(ring)))
    S, k = g["S"], g["k"]
    picks = np.full((S, k), -1, np.int32)
    att = np.zeros(S, np.uint32)
    N.check(lib.csa_legacy_find(enc.handle, k, g["seed"], 0, S, 0, N.ptr(picks), N.ptr(att)))
    assert att.tolist() == g["attempts"]
    assert picks[:len(g["picks"])].tolist() == g["picks"]
    # the batch host API takes the same kernel once a ring is set
    panels = np.zeros((S, enc.W), np.uint64)
    counts = np.zeros(enc.n, np.int64)
    uniq = np.zeros(1, np.uint64)
    flags = N.CSA_WANT_PANELS | N.CSA_WANT_COUNTS | N.CSA_WANT_UNIQUE
    N.check(lib.csa_legacy_sample(enc.handle, k, g["seed"], 0, S, flags, 0, N.ptr(panels), N.ptr(counts), None,
                                  N.ptr(uniq), None))
    assert counts.tolist() == g["counts"]
    assert int(uniq[0]) == g["unique"]
    assert hashlib.sha256(panels.tobytes()).hexdigest() == g["panels_sha256"]
    # the Python surface (analysis.legacy_find_batch with the columns)
    A = pkg("analysis")
    L.seed(g["seed"])
    got = A.legacy_find_batch(inst.categories, inst.agents, k, 8, columns_data=cols,
                              check_same_address_columns=g["columns"])
    assert got == g["picks"][:8]
    N.check(lib.csa_instance_set_address(enc.handle, None))


@pytest.mark.parametrize("case", ADDR)
def test_address_find_random_sample_legacy_single_attempts(gpu_available, case):
    """find_random_sample_legacy(..., True, columns) at the golden's (panel, attempt) stream
    positions: SelectionError where the reference raised it, else the same picks, log lines,
    counters and people left."""
    g, cols = _load(case)
    P = pkg()
    L = pkg("legacy")
    inst = P.read_instance(*inst_paths(g["instance"]), g["k"])
    L.seed(g["seed"])
    for rec in g["single_attempts"]:
        L.STREAM.panel, L.STREAM.attempt = rec["panel"], rec["attempt"]
        cats, people = copy.deepcopy(inst.categories), copy.deepcopy(inst.agents)
        if rec["status"] == "SelectionError":
            with pytest.raises(L.SelectionError):
                L.find_random_sample_legacy(cats, people, cols, g["k"], True, g["columns"])
            continue
        sel, lines = L.find_random_sample_legacy(cats, people, cols, g["k"], True, g["columns"])
        assert list(sel) == rec["picks"]
        assert lines == rec["lines"]
        assert [[c, f, v["selected"], v["remaining"]] for c in cats for f, v in cats[c].items()] == rec["selected"]
        assert sorted(people) == rec["people_left"]
