"""XMIN's LEGACY caller (xmin.py:464-474) on the device vs the C oracle.

The reference loop calls legacy_find up to 3n times and returns the first panel
not in the portfolio; the oracle restatement below draws the same Philox panels
(coracle.draw) and scans them in order.  Result panel, the None case and the
number of panel indices consumed must all match.
"""
import itertools

import numpy as np
import pytest

from conftest import inst_paths, pkg
from oracle import coracle
from oracle.legacy_oracle import read_instance as oracle_read

pytestmark = pytest.mark.gpu


def _expected(name, k, seed, first, tries, portfolio_rows):
    o = oracle_read(*inst_paths(name), k)
    rc, panels, _, _ = coracle.draw(o, k, seed, first, tries)
    assert rc == 0
    member = {r.tobytes() for r in portfolio_rows}
    for j in range(tries):
        if panels[j].tobytes() not in member:
            return j, panels[j]
    return -1, None


def _setup(name, k, seed, first):
    P = pkg()
    X = pkg("xmin")
    inst = P.read_instance(*inst_paths(name), k)
    P.seed(seed)
    pkg("legacy").STREAM.take_panels(first)
    return P, X, inst


@pytest.mark.parametrize("chunk", [1, 4, 256])
def test_first_non_member_sf_e(gpu_available, chunk):
    name, k, seed, first = "sf_e_110", 110, 3, 1000
    P, X, inst = _setup(name, k, seed, first)
    o = oracle_read(*inst_paths(name), k)
    _, head, _, _ = coracle.draw(o, k, seed, first, 7)          # the first 7 draws are members
    _, far, _, _ = coracle.draw(o, k, seed, 10 ** 6, 20)         # plus unrelated panels
    enc = P.encode(inst.categories, inst.agents)
    portfolio = [frozenset(enc.agent_ids[p] for p in P.instance.unpack_panel(r, enc.n))
                 for r in np.concatenate([head, far])]
    tries = 3 * len(inst.agents)
    ej, epanel = _expected(name, k, seed, first, tries, np.concatenate([head, far]))
    assert ej == 7
    got = X._get_panel_not_in_portfolio_if_possible(inst.categories, inst.agents, k, portfolio, chunk=chunk)
    want = frozenset(enc.agent_ids[p] for p in P.instance.unpack_panel(epanel, enc.n))
    assert got == want
    assert pkg("legacy").STREAM.panel == first + ej + 1


def test_all_members_returns_none(gpu_available):
    name, k, seed, first = "couples_panel_from_twenty_people_no_constraints_2", 2, 5, 17
    P, X, inst = _setup(name, k, seed, first)
    portfolio = [frozenset(c) for c in itertools.combinations(list(inst.agents), 2)]
    assert X._get_panel_not_in_portfolio_if_possible(inst.categories, inst.agents, k, portfolio, chunk=8) is None
    assert pkg("legacy").STREAM.panel == first + 3 * len(inst.agents)


@pytest.mark.parametrize("missing", [0, 57, 123])
def test_one_missing_pair(gpu_available, missing):
    name, k, seed, first = "couples_panel_from_twenty_people_no_constraints_2", 2, 9, 400
    P, X, inst = _setup(name, k, seed, first)
    pairs = list(itertools.combinations(list(inst.agents), 2))
    portfolio = [frozenset(c) for i, c in enumerate(pairs) if i != missing]
    enc = P.encode(inst.categories, inst.agents)
    rows = X.pack_portfolio(enc, portfolio)
    tries = 3 * len(inst.agents)
    ej, epanel = _expected(name, k, seed, first, tries, rows)
    got = X._get_panel_not_in_portfolio_if_possible(inst.categories, inst.agents, k, portfolio, chunk=4)
    if ej < 0:
        assert got is None
        assert pkg("legacy").STREAM.panel == first + tries
    else:
        assert got == frozenset(pairs[missing])
        assert got == frozenset(enc.agent_ids[p] for p in P.instance.unpack_panel(epanel, enc.n))
        assert pkg("legacy").STREAM.panel == first + ej + 1


def test_empty_portfolio_takes_first_panel(gpu_available):
    name, k, seed, first = "example_small_20", 20, 2, 0
    P, X, inst = _setup(name, k, seed, first)
    got = X._get_panel_not_in_portfolio_if_possible(inst.categories, inst.agents, k, [])
    P.seed(seed)
    assert got == frozenset(P.legacy_find(inst.categories, inst.agents, k))
    assert pkg("legacy").STREAM.panel == 1
