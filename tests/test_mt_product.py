"""MT19937 mode of the PRODUCT: csa_legacy_draw_mt in
libcsa_legacy.so (host code, csrc/legacy_mt.cpp), driven through legacy.mt_draw /
find_random_sample_legacy(rng="mt") with the stdlib random module's own state, against the
reference's PUBLISHED outputs (reference_output/ and analysis/ *_ratio_product_data.csv,
analysis/*_statistics.txt, committed in tests/golden/mt_published.json) and against the
reference's own check_same_address runs in MT mode (tests/golden/address_*.json, made by
tools/make_goldens.py).  No GPU: the MT draw is host code; the per-person counts here are
taken from the returned panels by the test.
"""
import copy
import json
import os
import random

import numpy as np
import pytest

from conftest import GOLD, inst_paths, pkg

with open(os.path.join(GOLD, "mt_published.json")) as fh:
    MT = json.load(fh)


def _counts(panels, n):
    bits = np.unpackbits(np.ascontiguousarray(panels).view(np.uint8), axis=1, bitorder="little")[:, :n]
    return bits.sum(axis=0, dtype=np.int64)


def _draw(name, k, S, seed):
    P = pkg()
    L = pkg("legacy")
    inst = P.read_instance(*inst_paths(name), k)
    enc = P.encode(inst.categories, inst.agents)
    random.seed(seed)                               # analysis.py:169
    picks, panels, attempts = L.mt_draw(enc, k, S)
    return enc, picks, panels, attempts


@pytest.mark.parametrize("rel", sorted(r for r in MT if r.endswith(".csv")))
def test_mt_seed0_matches_published(rel):
    g = MT[rel]
    enc, _, panels, _ = _draw(g["instance"], g["k"], g["S"], 0)
    assert [c / g["S"] for c in _counts(panels, enc.n)] == g["selection_probability"]


@pytest.mark.parametrize("name", ["couples_panel_from_twenty_people_no_constraints_2", "example_small_20"])
def test_mt_seed1_statistics(name):
    pins = MT["statistics_seed1"][name]
    k = int(name.rsplit("_", 1)[1])
    enc, _, p0, _ = _draw(name, k, 10000, 0)
    enc, _, p1, _ = _draw(name, k, 10000, 1)
    assert len(np.unique(p1, axis=0)) == pins["unique"]
    c0, c1 = _counts(p0, enc.n), _counts(p1, enc.n)
    minimiser = min(range(enc.n), key=lambda i: c0[i])      # analysis.py:565-571
    assert "%.4f" % (c1[minimiser] / 10000) == pins["minimizer_prop"]


def test_mt_state_is_the_stdlib_stream():
    """Pick orders equal the oracle's MT restatement (random.Random(seed).randint at every argmax
    improvement), and the global random state afterwards equals that generator's state: the draw
    consumed exactly the reference's randint words."""
    from oracle.legacy_oracle import MtRng, legacy_find, read_instance
    name, k, S, seed = "sf_e_tight_110", 110, 120, 5
    enc, picks, _, attempts = _draw(name, k, S, seed)
    after = random.getstate()
    o = read_instance(*inst_paths(name), k)
    src = MtRng(seed)
    want = [legacy_find(o, k, src, i) for i in range(S)]
    assert [list(map(int, row)) for row in picks] == [w[0] for w in want]
    assert attempts.tolist() == [w[1] for w in want]
    assert after == src.r.getstate()


ADDR = sorted(f[:-5] for f in os.listdir(GOLD) if f.startswith("address_") and f.endswith(".json"))


def _address_golden(case):
    with open(os.path.join(GOLD, case + ".json")) as fh:
        return json.load(fh)


def _columns(g, n):
    import csv
    path = os.path.join(os.path.dirname(GOLD), "..", g["addresses"])
    with open(path, encoding="utf-8") as fh:
        return {i: dict(r) for i, r in enumerate(csv.DictReader(fh))}


@pytest.mark.parametrize("case", ADDR)
def test_mt_same_address_legacy_find(case):
    """legacy_find semantics (restarts) with check_same_address, MT mode: pick orders and attempt
    counts equal the reference's own run (address golden, "mt")."""
    g = _address_golden(case)["mt"]
    P = pkg()
    L = pkg("legacy")
    inst = P.read_instance(*inst_paths(g["instance"]), g["k"])
    enc = P.encode(inst.categories, inst.agents)
    cols = _columns(g, enc.n)
    ring = L.address_rings(enc.agent_ids, cols, g["columns"])
    random.seed(g["seed"])
    picks, panels, attempts = L.mt_draw(enc, g["k"], g["S"], addr_next=ring)
    assert attempts.tolist() == g["attempts"]
    assert [list(map(int, r)) for r in picks[:len(g["picks"])]] == g["picks"]
    assert _counts(panels, enc.n).tolist() == g["counts"]


@pytest.mark.parametrize("case", ADDR)
def test_mt_find_random_sample_legacy_single_attempts(case):
    """find_random_sample_legacy(..., True, columns, rng="mt") attempt by attempt: SelectionError
    where the reference raised it, else the same picks, output lines, counters and people left."""
    g = _address_golden(case)["mt"]
    P = pkg()
    L = pkg("legacy")
    inst = P.read_instance(*inst_paths(g["instance"]), g["k"])
    cols = _columns(g, len(inst.agents))
    random.seed(g["seed"])
    for rec in g["single_attempts"]:
        cats, people = copy.deepcopy(inst.categories), copy.deepcopy(inst.agents)
        if rec["status"] == "SelectionError":
            with pytest.raises(L.SelectionError):
                L.find_random_sample_legacy(cats, people, cols, g["k"], True, g["columns"], rng="mt")
            continue
        sel, lines = L.find_random_sample_legacy(cats, people, cols, g["k"], True, g["columns"], rng="mt")
        assert list(sel) == rec["picks"]
        assert lines == rec["lines"]
        assert [[c, f, v["selected"], v["remaining"]] for c in cats for f, v in cats[c].items()] == rec["selected"]
        assert sorted(people) == rec["people_left"]


def test_mt_no_address_lines_match_reference_format():
    """Without check_same_address the lines are "Using legacy algorithm." plus one "Category ...
    full" line per cascade, as legacy.py:119 formats them."""
    P = pkg()
    L = pkg("legacy")
    inst = P.read_instance(*inst_paths("sf_e_110"), 110)
    random.seed(3)
    cats, people = copy.deepcopy(inst.categories), copy.deepcopy(inst.agents)
    sel, lines = L.find_random_sample_legacy(cats, people, {}, 110, False, [], rng="mt")
    assert lines[0] == "Using legacy algorithm." and len(sel) == 110
    assert all(ln.startswith("Category ") and " full - deleted " in ln for ln in lines[1:])
    assert len(people) == len(inst.agents) - 110 - sum(int(ln.split("deleted ")[1].split(",")[0]) for ln in lines[1:])


def test_mt_xmin_caller_consumes_like_the_reference():
    """XMIN's caller in MT mode: one legacy_find per try from the stdlib stream, the first panel not
    in the portfolio; the stream position afterwards equals drawing the same number of panels."""
    P = pkg()
    L = pkg("legacy")
    X = pkg("xmin")
    inst = P.read_instance(*inst_paths("couples_panel_from_twenty_people_no_constraints_2"), 2)
    enc = P.encode(inst.categories, inst.agents)
    random.seed(9)
    picks, _, _ = L.mt_draw(enc, 2, 6)
    panels = [frozenset(int(p) for p in row) for row in picks]
    portfolio = list(dict.fromkeys(panels[:5]))               # the first five draws are members
    random.seed(9)
    got = X._get_panel_not_in_portfolio_if_possible(inst.categories, inst.agents, 2, portfolio, rng="mt")
    want = next(p for p in panels if p not in portfolio)
    assert got == want
    after = random.getstate()
    random.seed(9)
    L.mt_draw(enc, 2, panels.index(want) + 1)
    assert random.getstate() == after
