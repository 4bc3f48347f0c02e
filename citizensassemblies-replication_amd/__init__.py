"""MI355X-native LEGACY Monte Carlo engine (citizens'-assembly replication hot path).

The package directory name contains a hyphen, so import it with
``importlib.import_module("citizensassemblies-replication_amd")`` (or add the
directory to ``sys.path``).  Public surface, mirroring the
reference's legacy.py / analysis.py LEGACY functions:

    read_instance, Instance, PairHistogram, SelectionError, check_min_cats,
    find_random_sample_legacy, legacy_find, legacy_probabilities, seed

plus set_rng_mode("mt" | "philox") (the reference's own MT19937 stream on the host, or the
device's Philox verification-mode stream, the default)

plus xmin._get_panel_not_in_portfolio_if_possible (XMIN's LEGACY caller,
xmin.py:464-474) on the device.
"""
from .instance import Instance, read_instance, encode  # noqa: F401
from .legacy import SelectionError, check_min_cats, find_random_sample_legacy, seed, set_rng_mode  # noqa: F401
from .analysis import PairHistogram, PanelSet, legacy_find, legacy_find_batch, legacy_probabilities  # noqa: F401
from . import _native, xmin  # noqa: F401

__all__ = ["Instance", "read_instance", "encode", "SelectionError", "check_min_cats",
           "find_random_sample_legacy", "seed", "set_rng_mode", "PairHistogram", "PanelSet", "legacy_find",
           "legacy_find_batch", "legacy_probabilities"]
