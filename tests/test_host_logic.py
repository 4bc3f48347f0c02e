"""Host-side logic on CPU: instance encoding, PairHistogram semantics, sharding helpers."""
import pickle

import numpy as np
import pytest

from conftest import pkg, inst_paths
from oracle.legacy_oracle import read_instance as oracle_read


@pytest.mark.parametrize("name,k", [("example_small_20", 20), ("sf_e_110", 110), ("pathological_5", 5)])
def test_encoding_matches_oracle_reader(name, k):
    P = pkg()
    inst = P.read_instance(*inst_paths(name), k)
    enc = P.encode(inst.categories, inst.agents)
    o = oracle_read(*inst_paths(name), k)
    assert enc.person_feat.tolist() == o.person_feat
    assert enc.fmin.tolist() == o.fmin and enc.fmax.tolist() == o.fmax and enc.fcat.tolist() == o.fcat
    assert enc.pool.tolist() == o.pool_counts()
    assert enc.rem0.tolist() == o.pool_counts()           # read_instance's "remaining" (analysis.py:136)
    assert enc.agent_ids == list(range(o.n))


def test_check_quotas_asserts():
    P = pkg()
    inst = P.read_instance(*inst_paths("example_small_20"), 20)
    enc = P.encode(inst.categories, inst.agents)
    enc.check_quotas(20)
    with pytest.raises(AssertionError):
        enc.check_quotas(500)        # sum(max) < k (analysis.py:176)


def _dict_hist(n):
    return {(i, j): 0 for i in range(n) for j in range(i + 1, n)}


def test_pair_histogram_semantics():
    A = pkg("analysis")
    n = 7
    h = A.PairHistogram(n)
    ref = _dict_hist(n)
    portfolio = [[0, 3, 5], [6, 1, 3], [2, 4]]
    h.add_portfolio_of_panels_to_histogram(portfolio, [1, 1, 1])
    for panel in portfolio:
        panel = list(panel)
        for a in range(len(panel)):
            for b in range(a + 1, len(panel)):
                key = tuple(sorted((panel[a], panel[b])))
                ref[key] += 1
    assert h.get_dict() == ref
    assert list(h.get_dict()) == list(ref)                 # row-major key order (analysis.py:70)
    assert h[(3, 0)] == h[(0, 3)] == 1
    h[(5, 0)] = 4
    assert h[(0, 5)] == 4
    h.turn_into_probabilities_by_dividing_all_elements_by_given_number(3)
    ref[(0, 5)] = 4
    assert h.get_dict() == {kk: v / 3 for kk, v in ref.items()}
    h2 = pickle.loads(pickle.dumps(h))
    assert h2.get_dict() == h.get_dict()
    u = A.PairHistogram(n, uniform_distribution=True)
    assert set(u.get_dict().values()) == {1 / (n * (n - 1) // 2)}


def test_pair_histogram_from_counts():
    A = pkg("analysis")
    m = np.arange(16, dtype=np.int64).reshape(4, 4)
    h = A.PairHistogram(4, counts=m)
    assert h[(2, 1)] == 6 and h[(0, 3)] == 3
    assert h.upper().tolist() == [1, 2, 3, 6, 7, 11]


def test_pair_histogram_divisors():
    """a zero divisor raises ZeroDivisionError as the reference's `/` does (analysis.py:86-88);
    negative and fractional divisors divide like the reference, pending or applied, host counts or not."""
    A = pkg("analysis")
    m = np.arange(16, dtype=np.int64).reshape(4, 4)
    ref = {(i, j): int(m[i, j]) for i in range(4) for j in range(i + 1, 4)}
    for div in (0, 0.0):
        h = A.PairHistogram(4, counts=m)
        with pytest.raises(ZeroDivisionError):
            h.turn_into_probabilities_by_dividing_all_elements_by_given_number(div)
        with pytest.raises(ZeroDivisionError):
            A.PairHistogram(4).turn_into_probabilities_by_dividing_all_elements_by_given_number(div)
    A.PairHistogram(1).turn_into_probabilities_by_dividing_all_elements_by_given_number(0)   # no pairs: no division
    for divs in ([-4], [2.5], [-3, 7], [10 ** 30]):
        h = A.PairHistogram(4, counts=m)
        for d in divs:
            h.turn_into_probabilities_by_dividing_all_elements_by_given_number(d)
        want = dict(ref)
        for d in divs:
            want = {kk: v / d for kk, v in want.items()}
        assert h.get_dict() == want


def test_shard_range_covers_exactly():
    D = pkg("distributed")
    for S in (0, 1, 7, 10000, 10 ** 6 + 3):
        for world in (1, 2, 3, 4, 8):
            prev = 0
            for r in range(world):
                b, e = D.shard_range(S, world, r)
                assert b == prev and e >= b
                prev = e
            assert prev == S


def test_owner_partition_dedupe():
    """Distinct panels summed over owner segments (owner = h1 % world) == the global count, for any
    world: equal panels have equal hashes, so they always meet at one owner."""
    D = pkg("distributed")
    rng = np.random.default_rng(0)
    p = rng.integers(0, 2 ** 63, size=(500, 4), dtype=np.int64).astype(np.uint64)
    p = np.concatenate([p, p[:100]])                       # 100 duplicates
    h = D.panel_hashes(p)
    for world in (1, 2, 4, 7):
        # the 600 panels split over `world` sender ranks, each sending its local distinct panels to
        # their owners; owner r's count over the segments from every sender
        shards = np.array_split(np.arange(len(p)), world)
        cap = D.exchange_capacity(max(len(x) for x in shards), world)
        segs = [D.segment_buckets(h[x], p[x], world, cap) for x in shards]
        total = 0
        for r in range(world):
            rh = np.stack([sg[0][r] for sg in segs])
            rp = np.stack([sg[1][r] for sg in segs])
            rc = np.array([sg[2][r] for sg in segs])
            total += D.distinct_segments(rh, rp, rc)
        assert total == 500


def test_legacy_stream_positions():
    L = pkg("legacy")
    s = L.LegacyStream(5)
    assert s.take_panels(10) == 0 and s.panel == 10
    assert s.take_attempt() == (10, 0) and s.take_attempt() == (10, 1)
    assert s.take_panels(1) == 10 and s.attempt == 0
    s.seed(1)
    assert (s.key, s.panel) == (1, 0)


def test_check_min_cats():
    L = pkg("legacy")
    cats = {"g": {"f": {"min": 1, "max": 2, "selected": 1, "remaining": 0},
                  "m": {"min": 2, "max": 2, "selected": 1, "remaining": 3}}}
    ok, msg = L.check_min_cats(cats)
    assert not ok and msg == ["Failed to get minimum in category: m"]
    cats["g"]["m"]["selected"] = 2
    assert L.check_min_cats(cats) == (True, [])


def test_pack_portfolio_roundtrip():
    """xmin.pack_portfolio: agent-id panels -> bitmask rows (unknown agents drop the panel)."""
    P = pkg()
    X = pkg("xmin")
    inst = P.read_instance(*inst_paths("example_small_20"), 20)
    enc = P.encode(inst.categories, inst.agents)
    ids = list(inst.agents)
    panels = [frozenset(ids[3:23]), frozenset(ids[150:170]), frozenset(ids[:19] + ["nobody"])]
    rows = X.pack_portfolio(enc, panels)
    assert rows.shape == (2, enc.W)
    for r, pnl in zip(rows, panels[:2]):
        assert frozenset(enc.agent_ids[p] for p in P.instance.unpack_panel(r, enc.n)) == pnl


def _oracle_raw(name, k, S, seed):
    from oracle import coracle
    A = pkg("analysis")
    inst = pkg().read_instance(*inst_paths(name), k)
    o = oracle_read(*inst_paths(name), k)
    rc, panels, _, _ = coracle.draw(o, k, seed, 0, S)
    assert rc == 0
    raw = A.LegacyRaw(coracle.counts(panels, o.n), coracle.pairs(panels, o.n), coracle.unique(panels, o.n),
                      panels, None)
    return inst, raw


@pytest.mark.parametrize("keep_panels", [True, False])
def test_legacy_cache_npz_roundtrip(tmp_path, keep_panels):
    """cache.save_legacy_npz / load_legacy_npz (run_legacy_or_retrieve, analysis.py:271-293):
    a retrieved result equals the freshly finished one bit for bit."""
    A = pkg("analysis")
    Cc = pkg("cache")
    S, seed = 3000, 0
    inst, raw = _oracle_raw("sf_e_110", 110, S, seed)
    enc = pkg().encode(inst.categories, inst.agents)
    alloc, found, hist = A.finish(inst, enc, raw, S)
    path = Cc.legacy_cache_path("sf_e_110", 110, False, tmp_path)
    assert path.name == "sf_e_110_110_legacy_first.npz"
    Cc.save_legacy_npz(path, enc, raw, S, seed, 110, keep_panels=keep_panels)
    alloc2, found2, hist2 = Cc.load_legacy_npz(path, inst)
    assert alloc2 == alloc
    assert len(found2) == len(found) == raw.unique
    assert np.array_equal(hist2.upper(), hist.upper())
    assert hist2.get_dict() == hist.get_dict()
    if keep_panels:
        assert set(found2) == set(found)


def test_legacy_cache_rejects_other_instance(tmp_path):
    Cc = pkg("cache")
    inst, raw = _oracle_raw("example_small_20", 20, 500, 1)
    enc = pkg().encode(inst.categories, inst.agents)
    path = tmp_path / "x.npz"
    Cc.save_legacy_npz(path, enc, raw, 500, 1, 20)
    other = pkg().read_instance(*inst_paths("sf_e_110"), 110)
    with pytest.raises(ValueError):
        Cc.load_legacy_npz(path, other)


@pytest.mark.parametrize("inst", ["example_small_20", "example_large_200",
                                  "couples_panel_from_twenty_people_no_constraints_2"])
def test_published_legacy_statistics(inst):
    """stats.compute_prob_allocation_stats / upper_confidence_bound on the reference's published
    seed-0 LEGACY allocations (tests/golden/mt_published.json) print the reference's published
    statistics lines (analysis.py:568-597; tests/golden/published_stats.json)."""
    import json
    import os
    from conftest import GOLD
    St = pkg("stats")
    pub = json.load(open(os.path.join(GOLD, "published_stats.json")))[inst]
    mt = json.load(open(os.path.join(GOLD, "mt_published.json")))[pub["alloc_key"]]
    alloc = dict(enumerate(mt["selection_probability"]))
    st = St.compute_prob_allocation_stats(alloc, True)
    assert f"{st.gini:.1%}" == pub["gini"]
    assert f"{st.geometric_mean:.1%}" == pub["geometric_mean"]
    assert f"{St.upper_confidence_bound(10000, float(pub['minimizer_prop'])):.2%}" == pub["ucb"]


def test_sorted_counts_to_probabilities():
    St = pkg("stats")
    rng = np.random.default_rng(3)
    counts = rng.integers(0, 50, 1000)
    hist = np.bincount(counts, minlength=60).astype(np.uint64)
    S = 977
    assert St.sorted_counts_to_probabilities(hist, S).tolist() == sorted((c / S for c in counts.tolist()))


def test_encode_cached_revalidates():
    """instance.encode_cached: same dicts -> same encoding; changed counters / agents -> new one."""
    import copy
    I = pkg("instance")
    inst = pkg().read_instance(*inst_paths("example_small_20"), 20)
    cats, agents = copy.deepcopy(inst.categories), dict(inst.agents)
    e1 = I.encode_cached(cats, agents)
    assert I.encode_cached(cats, agents) is e1
    assert I.encode_cached(copy.deepcopy(cats), agents) is not e1       # other dict object
    first = next(iter(cats))
    feat = next(iter(cats[first]))
    cats[first][feat]["selected"] += 1
    e2 = I.encode_cached(cats, agents)
    assert e2 is not e1 and int(e2.sel0.sum()) == 1
    del agents[0]
    e3 = I.encode_cached(cats, agents)
    assert e3 is not e2 and e3.n == 199


def test_result_tuple_pickles_host_only():
    """PanelSet / PairHistogram pickle as host data (analysis.py:284-290 dumps the returned tuple):
    the distinct panels travel as packed rows, the histogram as its divided matrix."""
    A = pkg("analysis")
    rng = np.random.default_rng(3)
    n, S = 70, 500
    panels = np.zeros((S, 2), np.uint64)
    for i in range(S):
        for p in rng.choice(n, size=5, replace=False):
            panels[i, p >> 6] |= np.uint64(1) << np.uint64(p & 63)
    panels[1] = panels[0]                      # a duplicate
    ids = list(range(100, 100 + n))            # agent ids are not bit positions
    want = {tuple(ids[p] for p in range(n) if (int(r[p >> 6]) >> (p & 63)) & 1) for r in panels}
    ps = A.PanelSet(len(want), panels, n, ids)
    counts = np.zeros((n, n), np.int64)
    counts[np.triu_indices(n, 1)] = rng.integers(0, 9, size=n * (n - 1) // 2)
    hist = A.PairHistogram(n, counts=counts)
    hist.turn_into_probabilities_by_dividing_all_elements_by_given_number(S)
    ps2, hist2 = pickle.loads(pickle.dumps((ps, hist)))
    assert len(ps2) == len(want) and set(ps2) == want
    assert ps2.rows().shape == (len(want), 2)
    assert np.array_equal(hist2.upper(), counts[np.triu_indices(n, 1)] / S)
    assert set(pickle.loads(pickle.dumps(ps2))) == want       # a materialised set pickles too
    empty = pickle.loads(pickle.dumps(A.PanelSet(7, None, n, ids)))
    assert len(empty) == 7
    with pytest.raises(RuntimeError):
        iter(empty)


def _xt_network(X):
    """Numpy model of xt_count_kernel's register transpose (csrc/csa_legacy.hip, wave_transpose64):
    the same v_perm selectors, lane swaps, DPP patterns, rotations and keep masks, lane by lane."""
    M = 0xFFFFFFFF
    lane = np.arange(64)
    lo = [int(x) & M for x in X]
    hi = [int(x) >> 32 for x in X]

    def perm(s0, s1, sel):
        out = []
        for i in range(64):
            v = (s0[i] << 32) | s1[i]
            sl = sel[i] if isinstance(sel, list) else sel
            out.append(sum(((v >> (8 * ((sl >> (8 * k)) & 0xFF))) & 0xFF) << (8 * k) for k in range(4)))
        return out

    def rot(y, r):
        return [((y[i] >> r[i]) | (y[i] << (32 - r[i]))) & M for i in range(64)]

    def move(x, f):
        return [x[f(i)] for i in range(64)]

    # s = 32: permlane32_swap(lo, hi): lanes 32-63 of lo <-> lanes 0-31 of hi
    lo, hi = lo[:32] + hi[:32], lo[32:] + hi[32:]
    # s = 16: gather, permlane16_swap (odd rows of A <-> even rows of B), re-interleave
    A, B = perm(hi, lo, 0x05040100), perm(hi, lo, 0x07060302)
    A2, B2 = A[:], B[:]
    for r in (0, 32):
        A2[r + 16:r + 32], B2[r:r + 16] = B[r:r + 16], A[r + 16:r + 32]
    lo, hi = perm(B2, A2, 0x05040100), perm(B2, A2, 0x07060302)
    # s = 8: lane-dependent byte gather, row_ror:8, lane-dependent merges
    b3 = [(i >> 3) & 1 for i in range(64)]
    sel = lambda one, zero: [one if b else zero for b in b3]  # noqa: E731
    R = move(perm(hi, lo, sel(0x06040200, 0x07050301)), lambda i: (i & ~15) | ((i + 8) & 15))
    lo, hi = perm(R, lo, sel(0x03050104, 0x05020400)), perm(R, hi, sel(0x03070106, 0x07020600))
    for s, keep0, f in ((4, 0x0F0F0F0F, lambda i: i ^ 4),
                        (2, 0x33333333, lambda i: i ^ 2), (1, 0x55555555, lambda i: i ^ 1)):
        bit = (lane // s) & 1
        keep = [(~keep0 & M) if b else keep0 for b in bit]
        r = [s if b else 32 - s for b in bit]
        out = []
        for h in (lo, hi):
            t = rot(move(h, f), r)
            out.append([(keep[i] & h[i]) | (~keep[i] & M & t[i]) for i in range(64)])
        lo, hi = out
    return [(hi[i] << 32) | lo[i] for i in range(64)]


def test_xt_register_transpose_network():
    import os
    import re
    rng = np.random.default_rng(7)
    X = rng.integers(0, 2 ** 63, size=64, dtype=np.uint64) | (rng.integers(0, 2, 64, dtype=np.uint64) << np.uint64(63))
    Y = _xt_network(X)
    bits = np.array([[(int(X[i]) >> j) & 1 for j in range(64)] for i in range(64)])
    tb = np.array([[(Y[j] >> i) & 1 for i in range(64)] for j in range(64)])
    assert (bits.T == tb).all()
    # DPP lane ^ 4 = quad_perm [3,2,1,0] (^3) then row_half_mirror (7 - i within 8 lanes)
    assert all(((i & ~7) | (7 - ((i ^ 3) & 7))) == i ^ 4 for i in range(64))
    # the model's constants are the kernel's
    src = open(os.path.join(os.path.dirname(__file__), "..", "citizensassemblies-replication_amd", "csrc",
                            "csa_legacy.hip")).read()
    body = src[src.index("__device__ __forceinline__ XtLane xt_lane_consts"):src.index("constexpr int kXtCols")]
    for c in ("0x05040100u", "0x07060302u", "0x06040200u", "0x07050301u", "0x03050104u", "0x05020400u",
              "0x03070106u", "0x07020600u", "0xF0F0F0F0u", "0x0F0F0F0Fu", "0xCCCCCCCCu", "0x33333333u",
              "0xAAAAAAAAu", "0x55555555u", "xt_dpp<0x128>", "xt_dpp<0x141>(xt_dpp<0x1B>", "xt_dpp<0x4E>",
              "xt_dpp<0xB1>"):
        assert c in body, c
    assert re.search(r"c\.r4 = b2 \? 4u : 28u", body)


def test_chunk_plan_rounds():
    """device.chunk_plan: chunks sum to S, stay <= C, are whole rounds except the last (one round
    before it), and fall back to equal cuts without a round size."""
    D = pkg("device")
    R = 131072
    assert D.chunk_plan(10 ** 6, 1 << 20, R) == [786432, 131072, 82496]
    assert D.chunk_plan(1250000, 1 << 20, 262144) == [786432, 262144, 201424]
    assert D.chunk_plan(5, 1 << 20, R) == [5] and D.chunk_plan(0, 10, R) == []
    assert D.chunk_plan(10, 4, 0) == [4, 4, 2]
    rng = np.random.default_rng(5)
    for _ in range(200):
        S, R = int(rng.integers(1, 10 ** 8)), int(rng.integers(1, 300000))
        C = int(rng.integers(R, 4 * R + 2))
        sizes = D.chunk_plan(S, C, R)
        assert sum(sizes) == S and all(0 < c <= C for c in sizes)
        if S > R:
            assert sizes[-2] == R and all(c % R == 0 for c in sizes[:-1])


def test_encoding_handle_per_device(monkeypatch):
    """EncodedInstance.handle is the native instance on the CURRENT HIP device, created there on first use
    (csa_current_device): a sharded call that runs on its rank's GPU without changing the caller's device,
    and a later call on another device, never launch on an instance of another device.  A fake library
    stands in for the C ABI (no GPU here)."""
    import ctypes
    P = pkg()
    N = pkg("_native")
    state = {"dev": 0, "made": [], "destroyed": [], "set_state": []}

    class Fake:
        def csa_current_device(self, out):
            ctypes.cast(out, ctypes.POINTER(ctypes.c_int32))[0] = state["dev"]
            return 0

        def csa_instance_create(self, n, C, F, pf, fmin, fmax, fcat, out):
            h = 1000 + len(state["made"])
            state["made"].append((state["dev"], h))
            ctypes.cast(out, ctypes.POINTER(ctypes.c_void_p))[0] = h
            return 0

        def csa_instance_set_state(self, h, sel, rem, present):
            state["set_state"].append(h.value)
            return 0

        def csa_instance_destroy(self, h):
            state["destroyed"].append(h.value)

    monkeypatch.setattr(N, "lib", lambda: Fake())
    cats = {"c": {"a": {"min": 0, "max": 2, "selected": 1}, "b": {"min": 0, "max": 2}}}
    enc = P.encode(cats, {0: {"c": "a"}, 1: {"c": "b"}})
    h0 = enc.handle
    assert enc.handle.value == h0.value and len(state["made"]) == 1      # cached on device 0
    state["dev"] = 3
    h3 = enc.handle
    assert h3.value != h0.value and state["made"][-1] == (3, h3.value)   # a new instance on device 3
    state["dev"] = 0
    assert enc.handle.value == h0.value and len(state["made"]) == 2
    assert state["set_state"] == [h0.value, h3.value]                    # the dicts' start state on each
    enc.close()
    assert sorted(state["destroyed"]) == sorted([h0.value, h3.value])
