"""GPU parity of every draw-kernel layout against the C oracle (Philox verification mode).

The batch path picks draw_batch_kernel (G = 4 / 8 lanes per panel) or draw_kernel
(G = 16 / 64) from the instance shape; CSA_DRAW_GROUP forces a layout.  Each must
give the oracle's panels and attempt counts bit-exactly, including the edge cases
of legacy.py:124-200 (restarts, rejections, max = 0 features, max = 0 < min).
"""
import os

import numpy as np
import pytest

from conftest import inst_paths, pkg
from oracle import coracle
from oracle.legacy_oracle import OracleInstance, read_instance as oracle_read

pytestmark = pytest.mark.gpu


@pytest.fixture
def draw_group():
    """Force a draw layout: an int G selects CSA_DRAW_GROUP=G (batch / general kernels, 1 = lane
    kernel with one lane per panel); "2L" / "4L" select the lane kernel with 2 / 4 lanes per panel
    (CSA_DRAW_LANE)."""
    names = ("CSA_DRAW_GROUP", "CSA_DRAW_LANE")
    old = {k: os.environ.get(k) for k in names}

    def set_layout(g):
        for k in names:
            os.environ.pop(k, None)
        if isinstance(g, str) and g.endswith("L"):
            os.environ["CSA_DRAW_LANE"] = g[:-1]
        else:
            os.environ["CSA_DRAW_GROUP"] = str(g)
    yield set_layout
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def _sample(enc, k, S, seed, begin=0, max_attempts=0):
    N = pkg("_native")
    panels = np.zeros((S, enc.W), np.uint64)
    attempts = np.zeros(S, np.uint32)
    N.check(N.lib().csa_legacy_sample(enc.handle, k, seed, begin, S, N.CSA_WANT_PANELS, max_attempts,
                                      N.ptr(panels), None, None, None, N.ptr(attempts)))
    return panels, attempts


@pytest.mark.parametrize("group", [1, "2L", "4L", 4, 8, 16, 64])
@pytest.mark.parametrize("name,k,S,seed", [("sf_e_tight_110", 110, 3000, 5), ("pathological_5", 5, 4000, 2),
                                           ("rejecty_6", 6, 20000, 8), ("example_small_20", 20, 20000, 1),
                                           ("couples_panel_from_twenty_people_no_constraints_2", 2, 20000, 3)])
def test_draw_layouts_match_oracle(gpu_available, draw_group, group, name, k, S, seed):
    P = pkg()
    draw_group(group)
    inst = P.read_instance(*inst_paths(name), k)
    enc = P.encode(inst.categories, inst.agents)
    begin = 987654321
    panels, attempts = _sample(enc, k, S, seed, begin)
    o = oracle_read(*inst_paths(name), k)
    rc, opanels, oatt, _ = coracle.draw(o, k, seed, begin, S)
    assert rc == 0
    assert np.array_equal(attempts, oatt)
    assert np.array_equal(panels, opanels)


def _weird_instance():
    """Category 'a': a0 [1, 3], a1 [0, 0] (dead), a2 [0, 2]; category 'b': b0 [1, 0] (max 0 < min),
    b1 [0, 3], b2 [1, 3].  40 agents with features drawn from a fixed generator."""
    cats = {"a": {"a0": {"min": 1, "max": 3}, "a1": {"min": 0, "max": 0}, "a2": {"min": 0, "max": 2}},
            "b": {"b0": {"min": 1, "max": 0}, "b1": {"min": 0, "max": 3}, "b2": {"min": 1, "max": 3}}}
    rng = np.random.default_rng(11)
    agents = {i: {"a": "a%d" % rng.integers(0, 3), "b": "b%d" % rng.integers(0, 3)} for i in range(40)}
    return cats, agents


@pytest.mark.parametrize("group", [1, "2L", "4L", 4, 8, 16, 64])
def test_zero_max_features_match_oracle(gpu_available, draw_group, group):
    """max = 0 features (dead, and max = 0 < min which routes to draw_kernel) vs the oracle."""
    P = pkg()
    draw_group(group)
    cats, agents = _weird_instance()
    k = 4
    enc = P.encode(cats, agents)
    feats = [(c, f) for c in cats for f in cats[c]]
    o = OracleInstance(k=k, cat_names=list(cats), feat_names=feats,
                       fmin=[cats[c][f]["min"] for c, f in feats], fmax=[cats[c][f]["max"] for c, f in feats],
                       fcat=[list(cats).index(c) for c, f in feats],
                       person_feat=[[feats.index(("a", agents[i]["a"])), feats.index(("b", agents[i]["b"]))]
                                    for i in range(40)])
    S, seed = 3000, 4
    rc, opanels, oatt, _ = coracle.draw(o, k, seed, 0, S, max_attempts=1000)
    panels, attempts = _sample(enc, k, S, seed, 0, max_attempts=1000)
    assert rc == 0
    assert np.array_equal(attempts, oatt)
    assert np.array_equal(panels, opanels)
