"""MT19937 mode of the oracle vs the reference's PUBLISHED LEGACY outputs.

reference_output/*_ratio_product_data.csv and analysis/*_ratio_product_data.csv
hold the seed-0, S=10,000 LEGACY selection probabilities in agent order
(analysis.py:441-447, 612); analysis/*_statistics.txt pin seed-1 quantities.
They are committed as data in tests/golden/mt_published.json.
"""
import json
import os

import pytest

from conftest import GOLD, inst_paths
from oracle.legacy_oracle import read_instance, legacy_probabilities

with open(os.path.join(GOLD, "mt_published.json")) as fh:
    MT = json.load(fh)


@pytest.mark.parametrize("rel", ["analysis/couples_panel_from_twenty_people_no_constraints_2_ratio_product_data.csv",
                                 "reference_output/example_small_20_ratio_product_data.csv",
                                 "analysis/example_small_20_ratio_product_data.csv"])
def test_mt_seed0_matches_published(rel):
    g = MT[rel]
    inst = read_instance(*inst_paths(g["instance"]), g["k"])
    res = legacy_probabilities(inst, g["S"], 0, mode="mt", want_pairs=False)
    assert [c / g["S"] for c in res.counts] == g["selection_probability"]


@pytest.mark.parametrize("name", ["couples_panel_from_twenty_people_no_constraints_2", "example_small_20"])
def test_mt_seed1_statistics(name):
    pins = MT["statistics_seed1"][name]
    k = int(name.rsplit("_", 1)[1])
    inst = read_instance(*inst_paths(name), k)
    first = legacy_probabilities(inst, 10000, 0, mode="mt", want_pairs=False)
    second = legacy_probabilities(inst, 10000, 1, mode="mt", want_pairs=False)
    assert second.unique == pins["unique"]
    # analysis.py:565-571: minimiser of the first sample, its proportion in the second
    minimiser = min(range(inst.n), key=lambda i: first.counts[i])
    assert "%.4f" % (second.counts[minimiser] / 10000) == pins["minimizer_prop"]
