"""GPU parity of every draw-kernel layout against the C oracle (Philox verification mode).

The batch path picks draw_solo_kernel (1 lane per panel), draw_lane_kernel (2 lanes per
panel) or draw_wide_kernel (8 lanes per panel, n up to 8192), all writing pick lists (packed
in the draw's tail or by picks_pack_kernel), or draw_kernel (G = 16 / 64) from the instance
shape; CSA_DRAW_KERNEL=solo|lane|wide|16|64 forces a layout the instance fits.  Each must give the
oracle's panels and attempt counts bit-exactly, including the edge cases of
legacy.py:124-200 (restarts, rejections, max = 0 features, max = 0 < min).
"""
import os

import numpy as np
import pytest

from conftest import PHILOX_CASES, golden, inst_paths, pkg
from oracle import coracle
from oracle.legacy_oracle import OracleInstance, read_instance as oracle_read

pytestmark = pytest.mark.gpu


@pytest.fixture
def draw_group():
    """Force a batch draw layout (CSA_DRAW_KERNEL = "solo" / "lane" / "wide" / "16" / "64")."""
    old = os.environ.get("CSA_DRAW_KERNEL")

    def set_layout(g):
        os.environ["CSA_DRAW_KERNEL"] = str(g)
    yield set_layout
    if old is None:
        os.environ.pop("CSA_DRAW_KERNEL", None)
    else:
        os.environ["CSA_DRAW_KERNEL"] = old


def _sample(enc, k, S, seed, begin=0, max_attempts=0):
    N = pkg("_native")
    panels = np.zeros((S, enc.W), np.uint64)
    attempts = np.zeros(S, np.uint32)
    N.check(N.lib().csa_legacy_sample(enc.handle, k, seed, begin, S, N.CSA_WANT_PANELS, max_attempts,
                                      N.ptr(panels), None, None, None, N.ptr(attempts)))
    return panels, attempts


@pytest.mark.parametrize("group", ["solo", "lane", "wide", 16, 64])
@pytest.mark.parametrize("name,k,S,seed", [("sf_e_tight_110", 110, 3000, 5), ("pathological_5", 5, 4000, 2),
                                           ("rejecty_6", 6, 20000, 8), ("example_small_20", 20, 20000, 1),
                                           ("couples_panel_from_twenty_people_no_constraints_2", 2, 20000, 3),
                                           ("synthetic8192_200", 200, 2000, 6)])
def test_draw_layouts_match_oracle(gpu_available, draw_group, group, name, k, S, seed):
    P = pkg()
    draw_group(group)
    inst = P.read_instance(*inst_paths(name), k)
    enc = P.encode(inst.categories, inst.agents)
    begin = 987654321
    A = pkg("analysis")
    A.draw_stats(enc, reset=True)
    panels, attempts = _sample(enc, k, S, seed, begin)
    stats = A.draw_stats(enc)
    o = oracle_read(*inst_paths(name), k)
    rejects = np.zeros(S, np.uint32)
    rc, opanels, oatt, _ = coracle.draw(o, k, seed, begin, S, rejects=rejects)
    assert rc == 0
    assert np.array_equal(attempts, oatt)
    assert np.array_equal(panels, opanels)
    # the kernel's restart counters (csa_instance_draw_stats) split like the oracle's
    assert stats == {"attempts": int(oatt.sum()), "rejections": int(rejects.sum()),
                     "selection_errors": int(oatt.sum()) - S - int(rejects.sum())}


def _weird_instance():
    """Category 'a': a0 [1, 3], a1 [0, 0] (dead), a2 [0, 2]; category 'b': b0 [1, 0] (max 0 < min),
    b1 [0, 3], b2 [1, 3].  40 agents with features drawn from a fixed generator."""
    cats = {"a": {"a0": {"min": 1, "max": 3}, "a1": {"min": 0, "max": 0}, "a2": {"min": 0, "max": 2}},
            "b": {"b0": {"min": 1, "max": 0}, "b1": {"min": 0, "max": 3}, "b2": {"min": 1, "max": 3}}}
    rng = np.random.default_rng(11)
    agents = {i: {"a": "a%d" % rng.integers(0, 3), "b": "b%d" % rng.integers(0, 3)} for i in range(40)}
    return cats, agents


@pytest.mark.parametrize("group", ["solo", "lane", "wide", 16, 64])
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


@pytest.mark.parametrize("name,k,S,seed", [("sf_e_tight_110", 110, 3000, 5), ("example_small_20", 20, 5000, 3),
                                           ("pathological_5", 5, 4000, 2), ("synthetic8192_200", 200, 3000, 4)])
def test_pick_lists_match_oracle_pick_order(gpu_available, name, k, S, seed):
    """csa_draw_picks_async writes each accepted panel's picks in pick order (the order of
    people_selected, legacy.py:194); csa_picks_pack_async packs them (+ hashes) bit-exactly."""
    import torch
    P = pkg()
    N = pkg("_native")
    D = pkg("distributed")
    inst = P.read_instance(*inst_paths(name), k)
    enc = P.encode(inst.categories, inst.agents)
    assert N.lib().csa_draw_picks_supported(enc.handle, k) == 1
    begin = 4242
    kp = int(N.lib().csa_picks_stride(k))
    picks = torch.empty(S * kp, dtype=torch.int16, device="cuda")
    att = torch.empty(S, dtype=torch.int32, device="cuda")
    status = torch.zeros(4, dtype=torch.int32, device="cuda")
    N.check(N.lib().csa_draw_picks_async(enc.handle, k, seed, begin, S, 0, N.ptr(picks), N.ptr(att), N.ptr(status),
                                         None))
    panels = torch.empty(S * enc.W, dtype=torch.int64, device="cuda")
    hashes = torch.empty(2 * S, dtype=torch.int64, device="cuda")
    N.check(N.lib().csa_picks_pack_async(N.ptr(picks), S, k, enc.n, N.ptr(panels), N.ptr(hashes), None))
    torch.cuda.synchronize()
    assert int(status[0].item()) == 0
    o = oracle_read(*inst_paths(name), k)
    rc, opanels, oatt, opicks = coracle.draw(o, k, seed, begin, S, want_picks=True)
    assert rc == 0
    assert np.array_equal(picks.cpu().numpy().astype(np.int32).reshape(S, kp)[:, :k], opicks)
    assert np.array_equal(att.cpu().numpy().astype(np.uint32), oatt)
    got = panels.cpu().numpy().view(np.uint64).reshape(S, enc.W)
    assert np.array_equal(got, opanels)
    assert np.array_equal(hashes.cpu().numpy().view(np.uint64).reshape(S, 2), D.panel_hashes(opanels))


@pytest.mark.parametrize("S", [1, 63, 64, 65, 1000, 4097])
def test_picks_pack_edges(gpu_available, S):
    """picks_pack_kernel on ragged batch tails and odd k (u32 loads of two picks, a single last
    pick), checked against a host packing of random distinct picks."""
    import torch
    N = pkg("_native")
    D = pkg("distributed")
    rng = np.random.default_rng(S)
    for n, k in ((200, 7), (1727, 110), (64, 1), (2048, 33)):
        kp = int(N.lib().csa_picks_stride(k))
        picks = np.full((S, kp), -1, np.int16)          # entries past k are ignored
        picks[:, :k] = np.stack([rng.choice(n, size=k, replace=False) for _ in range(S)])
        want = np.zeros((S, (n + 63) // 64), np.uint64)
        for i in range(S):
            for p in picks[i, :k].astype(np.int64):
                want[i, p >> 6] |= np.uint64(1) << np.uint64(p & 63)
        d = torch.from_numpy(picks.ravel().copy()).cuda()
        W = (n + 63) // 64
        panels = torch.full((S * W,), -1, dtype=torch.int64, device="cuda")
        hashes = torch.empty(2 * S, dtype=torch.int64, device="cuda")
        N.check(N.lib().csa_picks_pack_async(N.ptr(d), S, k, n, N.ptr(panels), N.ptr(hashes), None))
        torch.cuda.synchronize()
        assert np.array_equal(panels.cpu().numpy().view(np.uint64).reshape(S, W), want)
        assert np.array_equal(hashes.cpu().numpy().view(np.uint64).reshape(S, 2), D.panel_hashes(want))


def test_k_zero_draws_empty_panels(gpu_available):
    """k = 0 (legacy.py:184 loops zero times): empty panels accepted at the first attempt when no
    feature has min > 0, else the reference restarts forever -> attempt limit."""
    P = pkg()
    N = pkg("_native")
    cats = {"a": {"x": {"min": 0, "max": 2}, "y": {"min": 0, "max": 2}}}
    agents = {i: {"a": "x" if i % 2 else "y"} for i in range(10)}
    enc = P.encode(cats, agents)
    panels, attempts = _sample(enc, 0, 100, 3)
    assert not panels.any() and np.all(attempts == 1)
    cats["a"]["x"]["min"] = 1
    enc = P.encode(cats, agents)
    with pytest.raises(N.CsaError):
        _sample(enc, 0, 10, 3, max_attempts=5)


@pytest.mark.parametrize("group", ["solo", "lane"])
@pytest.mark.parametrize("case", PHILOX_CASES)
def test_register_layouts_match_goldens(gpu_available, draw_group, group, case):
    """The one- and two-lane register kernels (fused pack included) against the reference goldens."""
    import hashlib
    P = pkg()
    A = pkg("analysis")
    draw_group(group)
    g = golden(case)
    inst = P.read_instance(*inst_paths(g["instance"]), g["k"])
    enc = P.encode(inst.categories, inst.agents)
    raw = A.legacy_sample_raw(enc, g["k"], g["S"], g["seed"], want_pairs=False, want_panels=True,
                              want_attempts=True)
    assert hashlib.sha256(np.ascontiguousarray(raw.panels).tobytes()).hexdigest() == g["panels_sha256"]
    assert raw.attempts.tolist() == g["attempts"]
    assert raw.unique == g["unique"]


def _synthetic(F_per_cat, n, k, seed):
    """Random pool: categories with the given feature counts, shares ~ Dirichlet(2), quotas
    floor(0.9 k p) / ceil(1.1 k p) (the SURVEY §8(d) synthetic recipe)."""
    rng = np.random.default_rng(seed)
    cats, feats, fmin, fmax, fcat = {}, [], [], [], []
    shares = []
    for c, nf in enumerate(F_per_cat):
        p = rng.dirichlet(np.full(nf, 2.0))
        shares.append(p)
        cats["c%d" % c] = {}
        for j in range(nf):
            lo, hi = int(np.floor(0.9 * k * p[j])), int(np.ceil(1.1 * k * p[j]))
            cats["c%d" % c]["f%d" % j] = {"min": lo, "max": hi}
            feats.append(("c%d" % c, "f%d" % j))
            fmin.append(lo)
            fmax.append(hi)
            fcat.append(c)
    picks = [rng.choice(len(p), size=n, p=p) for p in shares]
    agents = {i: {"c%d" % c: "f%d" % picks[c][i] for c in range(len(F_per_cat))} for i in range(n)}
    pf = [[feats.index(("c%d" % c, "f%d" % picks[c][i])) for c in range(len(F_per_cat))] for i in range(n)]
    o = OracleInstance(k=k, cat_names=list(cats), feat_names=feats, fmin=fmin, fmax=fmax, fcat=fcat,
                       person_feat=pf)
    return cats, agents, o


@pytest.mark.parametrize("F_per_cat,n,k", [((4, 4, 4), 1800, 100),   # one-lane kernel FN = 16, WN = 32
                                           ((4, 4, 4), 1700, 100),   # FN = 16, WN = 28: 4 recount parts of 7 words
                                           ((3, 3), 1700, 120),      # FN = 8, WN = 28: 4 parts
                                           ((3, 3), 200, 30),        # FN = 8, WN = 4
                                           ((5, 5, 4), 100, 20)])    # FN = 16, WN = 4: one word per part
def test_one_lane_layouts_match_oracle(gpu_available, F_per_cat, n, k):
    """draw_solo_kernel's recount layouts (64/FN word parts, fewer where they do not divide WN)
    on synthetic pools the public instances do not cover, against the C oracle."""
    P = pkg()
    N = pkg("_native")
    cats, agents, o = _synthetic(F_per_cat, n, k, seed=n + k)
    enc = P.encode(cats, agents)
    buf = np.zeros(64, np.uint8)
    N.check(N.lib().csa_draw_kernel_name(enc.handle, k, buf.ctypes.data_as(__import__("ctypes").c_char_p), 64))
    assert bytes(buf).split(b"\0")[0].startswith(b"draw_solo_kernel")
    S, seed, begin = 4000, 3, 77
    rc, opanels, oatt, _ = coracle.draw(o, k, seed, begin, S, max_attempts=100000)
    panels, attempts = _sample(enc, k, S, seed, begin)
    assert rc == 0
    assert np.array_equal(attempts, oatt)
    assert np.array_equal(panels, opanels)


def _synthetic_tight(F_per_cat, n, k, seed, lo=0.9, hi=1.1):
    """As _synthetic with quotas floor(lo k p) / ceil(hi k p): lo, hi near 1 make restarts frequent."""
    rng = np.random.default_rng(seed)
    cats, feats, fmin, fmax, fcat, shares = {}, [], [], [], [], []
    for c, nf in enumerate(F_per_cat):
        p = rng.dirichlet(np.full(nf, 2.0))
        shares.append(p)
        cats["c%d" % c] = {}
        for j in range(nf):
            a, b = int(np.floor(lo * k * p[j])), int(np.ceil(hi * k * p[j]))
            cats["c%d" % c]["f%d" % j] = {"min": a, "max": b}
            feats.append(("c%d" % c, "f%d" % j))
            fmin.append(a)
            fmax.append(b)
            fcat.append(c)
    picks = [rng.choice(len(p), size=n, p=p) for p in shares]
    agents = {i: {"c%d" % c: "f%d" % picks[c][i] for c in range(len(F_per_cat))} for i in range(n)}
    pf = [[feats.index(("c%d" % c, "f%d" % picks[c][i])) for c in range(len(F_per_cat))] for i in range(n)]
    o = OracleInstance(k=k, cat_names=list(cats), feat_names=feats, fmin=fmin, fmax=fmax, fcat=fcat,
                       person_feat=pf)
    return cats, agents, o


@pytest.mark.parametrize("F_per_cat,n,k,lo,hi,want", [
    ((4, 4, 4, 4, 4), 3000, 120, 0.9, 1.1, "draw_wide_kernel<8, 4, 8>"),    # W = 47: 8 words per lane
    ((8,) * 8, 3900, 150, 0.9, 1.1, "draw_wide_kernel<8, 8, 8>"),          # F = 64: 8 features per lane
    ((6,) * 10, 8000, 200, 0.95, 1.05, "draw_wide_kernel<8, 8, 16>"),      # F = 60, W = 125, restarts
    ((3, 4, 5), 2500, 90, 0.97, 1.03, "draw_wide_kernel<8, 2, 8>"),        # F = 12 past the lane kernel's W
])
def test_wide_layouts_match_oracle(gpu_available, F_per_cat, n, k, lo, hi, want):
    """draw_wide_kernel's feature / word splits the public instances do not reach (FPL 2 / 4 / 8, WPL 8 /
    16, ragged last lanes), on synthetic pools against the C oracle: panels, attempts and the restart
    counters, through the default routing (n > 2048 or W > 32 takes the wide kernel)."""
    import ctypes
    P = pkg()
    N = pkg("_native")
    A = pkg("analysis")
    cats, agents, o = _synthetic_tight(F_per_cat, n, k, seed=n + k, lo=lo, hi=hi)
    enc = P.encode(cats, agents)
    buf = np.zeros(64, np.uint8)
    N.check(N.lib().csa_draw_kernel_name(enc.handle, k, buf.ctypes.data_as(ctypes.c_char_p), 64))
    assert bytes(buf).split(b"\0")[0].decode() == want
    S, seed, begin = 3000, 7, 5550001
    rejects = np.zeros(S, np.uint32)
    rc, opanels, oatt, _ = coracle.draw(o, k, seed, begin, S, max_attempts=100000, rejects=rejects)
    A.draw_stats(enc, reset=True)
    panels, attempts = _sample(enc, k, S, seed, begin, max_attempts=100000)
    stats = A.draw_stats(enc)
    assert rc == 0
    assert np.array_equal(attempts, oatt)
    assert np.array_equal(panels, opanels)
    assert stats == {"attempts": int(oatt.sum()), "rejections": int(rejects.sum()),
                     "selection_errors": int(oatt.sum()) - S - int(rejects.sum())}


@pytest.mark.parametrize("F_per_cat,n,k,lo,hi,wn", [
    ((6, 6, 6), 1000, 80, 0.9, 1.1, 16),      # F = 18, W = 16
    ((6, 6, 6), 1000, 90, 0.97, 1.03, 16),    # restarts
    ((8, 8, 8, 6), 1700, 110, 0.9, 1.1, 28),  # F = 30, W = 27 (the sf_e shape)
    ((8, 8, 8, 6), 1650, 100, 0.96, 1.04, 28),
])
def test_two_lane_layouts_match_oracle(gpu_available, F_per_cat, n, k, lo, hi, wn):
    """draw_lane_kernel through the default routing on synthetic pools with 16 < F <= 32 (W = 16 and the
    sf_e shape W = 26-27, with and without restarts), against the C oracle: panels, attempts and the
    restart counters."""
    import ctypes
    P = pkg()
    N = pkg("_native")
    A = pkg("analysis")
    cats, agents, o = _synthetic_tight(F_per_cat, n, k, seed=n + k, lo=lo, hi=hi)
    enc = P.encode(cats, agents)
    buf = np.zeros(64, np.uint8)
    N.check(N.lib().csa_draw_kernel_name(enc.handle, k, buf.ctypes.data_as(ctypes.c_char_p), 64))
    name = bytes(buf).split(b"\0")[0].decode()
    assert name.startswith("draw_lane_kernel<32, %d" % wn), name
    S, seed, begin = 2600, 9, 31337
    rejects = np.zeros(S, np.uint32)
    rc, opanels, oatt, _ = coracle.draw(o, k, seed, begin, S, max_attempts=100000, rejects=rejects)
    A.draw_stats(enc, reset=True)
    panels, attempts = _sample(enc, k, S, seed, begin, max_attempts=100000)
    stats = A.draw_stats(enc)
    assert rc == 0
    assert np.array_equal(attempts, oatt)
    assert np.array_equal(panels, opanels)
    assert stats == {"attempts": int(oatt.sum()), "rejections": int(rejects.sum()),
                     "selection_errors": int(oatt.sum()) - S - int(rejects.sum())}


@pytest.mark.parametrize("F_per_cat,n,k,lo,hi,kernel,k8", [
    ((8, 8, 8, 6), 1700, 110, 0.9, 1.1, "draw_lane_kernel<32, 28", True),
    ((6, 6, 6), 1900, 600, 0.93, 1.07, "draw_lane_kernel<32, 32", False),   # a min above 127
    ((3, 3), 1500, 300, 0.95, 1.05, "draw_solo_kernel<8, 28", False),
    ((3, 3), 1500, 90, 0.9, 1.1, "draw_solo_kernel<8, 28", True),
])
def test_key_width_variants_match_oracle(gpu_available, F_per_cat, n, k, lo, hi, kernel, k8):
    """The register kernels in both key widths: 8-bit need keys carrying the feature index (every
    need in [-127, 127], the BASELINE shapes) and the 16-bit keys an instance with a min above 127
    takes -- routing by csa_instance::need8 and panels / attempts / restart counters vs the C oracle."""
    import ctypes
    P = pkg()
    N = pkg("_native")
    A = pkg("analysis")
    cats, agents, o = _synthetic_tight(F_per_cat, n, k, seed=n + k + 1, lo=lo, hi=hi)
    assert (max(o.fmin) <= 127) == k8
    enc = P.encode(cats, agents)
    buf = np.zeros(64, np.uint8)
    N.check(N.lib().csa_draw_kernel_name(enc.handle, k, buf.ctypes.data_as(ctypes.c_char_p), 64))
    name = bytes(buf).split(b"\0")[0].decode()
    assert name.startswith(kernel) and name.endswith("true>" if k8 else "false>"), name
    S, seed, begin = 3000, 11, 4096
    rejects = np.zeros(S, np.uint32)
    rc, opanels, oatt, _ = coracle.draw(o, k, seed, begin, S, max_attempts=100000, rejects=rejects)
    A.draw_stats(enc, reset=True)
    panels, attempts = _sample(enc, k, S, seed, begin, max_attempts=100000)
    stats = A.draw_stats(enc)
    assert rc == 0
    assert np.array_equal(attempts, oatt)
    assert np.array_equal(panels, opanels)
    assert stats == {"attempts": int(oatt.sum()), "rejections": int(rejects.sum()),
                     "selection_errors": int(oatt.sum()) - S - int(rejects.sum())}
