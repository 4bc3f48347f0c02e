"""Pin the oracle: Python and C restatements vs vectors from the UNMODIFIED reference.

tests/golden/philox_*.json were produced by tools/make_goldens.py, which drives
/root/reference's legacy.py/analysis.py with only random.randint replaced by
the Philox verification-mode stream (no reference source is copied).
"""
import hashlib

import numpy as np
import pytest

from conftest import PHILOX_CASES, golden, inst_paths
from oracle import coracle
from oracle.legacy_oracle import read_instance, legacy_probabilities, pack_panels


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _load(g):
    c, r = inst_paths(g["instance"])
    return read_instance(c, r, g["k"])


@pytest.mark.parametrize("case", PHILOX_CASES)
def test_c_oracle_matches_reference(case):
    g = golden(case)
    inst = _load(g)
    rejects = np.zeros(g["S"], np.uint32)
    rc, panels, attempts, picks = coracle.draw(inst, g["k"], g["seed"], 0, g["S"], want_picks=True, rejects=rejects)
    assert rc == 0
    n = inst.n
    assert _sha(panels) == g["panels_sha256"]
    assert attempts.tolist() == g["attempts"]
    # restarts split as the reference raised them: SelectionErrors vs min-quota rejections
    assert rejects.tolist() == g["rejections"]
    assert (attempts - 1 - rejects).tolist() == g["selection_errors"]
    assert coracle.counts(panels, n).tolist() == g["counts"]
    assert coracle.unique(panels, n) == g["unique"]
    assert picks[: len(g["first_picks"])].tolist() == g["first_picks"]
    # pairs at every n, synthetic8192_200_s0 included (200 reference panels, 33.5 M pairs)
    pr = coracle.pairs(panels, n)
    up = pr[np.triu_indices(n, 1)]
    assert _sha(up) == g["pair_upper_sha256"]
    assert int(up.sum()) == g["pair_upper_sum"]
    # derived probabilities: the reference's own float64 pair values
    assert _sha(up / g["S"]) == g["pair_prob_sha256"]


@pytest.mark.parametrize("case", ["couples_s0", "couples_s1", "pathological_5_s0", "rejecty_6_s3",
                                  "sf_e_110_s0"])
def test_python_oracle_matches_reference(case):
    g = golden(case)
    inst = _load(g)
    S = min(g["S"], 2000)
    res = legacy_probabilities(inst, S, g["seed"], mode="philox")
    assert res.attempts == g["attempts"][:S]
    assert [list(p) for p in res.panels[:256]] == g["first_panels"][: min(S, 256)]
    assert res.picks[:64] == g["first_picks"][: min(S, 64)]
    if S == g["S"]:
        assert res.counts.tolist() == g["counts"]
        assert res.unique == g["unique"]
        assert _sha(pack_panels(res.panels, inst.n)) == g["panels_sha256"]


def test_alloc_floats_are_count_over_S():
    # the reference's alloc values are exactly count/S (analysis.py:190)
    for case in ("couples_s0", "example_small_20_s0"):
        g = golden(case)
        assert g["alloc"] == [c / g["S"] for c in g["counts"]]


def test_couples_known_answers():
    # every couples panel is 1 female + 1 male: same-sex pairs never co-occur
    g = golden("couples_s1")
    inst = _load(g)
    up = np.zeros((inst.n, inst.n), np.int64)
    up[np.triu_indices(inst.n, 1)] = g["pair_upper"]
    sex = [inst.person_feat[p][0] for p in range(inst.n)]
    for i in range(inst.n):
        for j in range(i + 1, inst.n):
            if sex[i] == sex[j]:
                assert up[i, j] == 0
    assert g["unique"] == 100
