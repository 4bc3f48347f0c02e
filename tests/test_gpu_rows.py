"""SURVEY.md section 8(f) rows 2-3 on the device: the LEGACY result cache
(run_legacy_or_retrieve, analysis.py:271-293) and the sorted pair-probability curve
(analysis.py:339-342) from pair_histogram_kernel, against the reference goldens and the
C oracle."""
import numpy as np
import pytest

from conftest import golden, inst_paths, pkg
from oracle import coracle
from oracle.legacy_oracle import read_instance as oracle_read

pytestmark = pytest.mark.gpu


def test_run_legacy_or_retrieve_golden(gpu_available, tmp_path):
    """First call draws on the GPU and writes the npz; the second call loads it.  Both equal the
    reference's own seed-0 result (tests/golden/philox_example_small_20_s0.json)."""
    Cc = pkg("cache")
    g = golden("example_small_20_s0")
    inst = pkg().read_instance(*inst_paths(g["instance"]), g["k"])
    for call in range(2):
        alloc, found, hist = Cc.run_legacy_or_retrieve("example_small_20", inst, False, directory=tmp_path,
                                                       iterations=g["S"])
        assert (tmp_path / "example_small_20_20_legacy_first.npz").exists()
        assert [alloc[i] for i in range(len(alloc))] == g["alloc"]
        assert len(found) == g["unique"]
        assert tuple(g["first_panels"][0]) in found
        assert hist.upper().tolist() == (np.asarray(g["pair_upper"]) / g["S"]).tolist()
        # the pair-curve consumer works on a retrieved result as on a fresh one
        assert pkg("stats").sorted_pair_probabilities(hist).tolist() == sorted(hist.upper().tolist())


def test_run_legacy_or_retrieve_resample_seed(gpu_available, tmp_path):
    """resample=True -> seed 1, file *_legacy_second.npz (analysis.py:282-284)."""
    Cc = pkg("cache")
    A = pkg("analysis")
    inst = pkg().read_instance(*inst_paths("sf_e_110"), 110)
    alloc, found, hist = Cc.run_legacy_or_retrieve("sf_e_110", inst, True, directory=tmp_path, iterations=3000)
    assert (tmp_path / "sf_e_110_110_legacy_second.npz").exists()
    alloc2, found2, hist2 = A.legacy_probabilities(inst, 3000, 1)
    assert alloc == alloc2 and len(found) == len(found2)
    assert np.array_equal(hist.upper(), hist2.upper())
    alloc3, found3, hist3 = Cc.run_legacy_or_retrieve("sf_e_110", inst, True, directory=tmp_path, iterations=3000)
    assert alloc3 == alloc and set(found3) == set(found) and np.array_equal(hist3.upper(), hist.upper())


@pytest.mark.parametrize("name,k,S,seed", [("example_small_20", 20, 10000, 0), ("sf_e_110", 110, 20000, 4),
                                           ("couples_panel_from_twenty_people_no_constraints_2", 2, 10000, 1)])
def test_sorted_pair_probabilities(gpu_available, name, k, S, seed):
    """Device histogram of the pair counts -> the reference's sorted(get_dict().values())."""
    A = pkg("analysis")
    St = pkg("stats")
    inst = pkg().read_instance(*inst_paths(name), k)
    _, _, hist = A.legacy_probabilities(inst, S, seed)
    got = St.sorted_pair_probabilities(hist)
    o = oracle_read(*inst_paths(name), k)
    rc, panels, _, _ = coracle.draw(o, k, seed, 0, S)
    pairs = coracle.pairs(panels, o.n)
    want = sorted((pairs[np.triu_indices(o.n, 1)] / S).tolist())
    assert got.tolist() == want
    assert got.tolist() == sorted(hist.get_dict().values())


def test_pair_histogram_overflow_and_edges(gpu_available):
    import torch
    St = pkg("stats")
    n = 300
    rng = np.random.default_rng(0)
    m = rng.integers(0, 40, (n, n)).astype(np.int64)
    d = torch.from_numpy(m).cuda()
    h = St.pair_count_histogram(d, n, 64)
    assert h.tolist() == np.bincount(m[np.triu_indices(n, 1)], minlength=64).tolist()
    with pytest.raises(ValueError):
        St.pair_count_histogram(d, n, 20)
    assert St.pair_count_histogram(d[:1], 1, 4).tolist() == [0, 0, 0, 0]
