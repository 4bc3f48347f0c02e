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


def test_hash_partition_dedupe():
    D = pkg("distributed")
    rng = np.random.default_rng(0)
    h = rng.integers(0, 2 ** 63, size=(500, 2), dtype=np.int64).astype(np.uint64)
    h = np.concatenate([h, h[:100]])                       # 100 duplicates
    total = sum(D.dedupe_hash_partition(h.ravel(), 4, r) for r in range(4))
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
