"""Shared fixtures.  `-m gpu` tests need an MI355X; everything else runs on CPU."""
import importlib
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(REPO, "tests", "golden")
INST = os.path.join(GOLD, "instances")
PKG_NAME = "citizensassemblies-replication_amd"
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) -- run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pkg(sub=None):
    return importlib.import_module(PKG_NAME + ("." + sub if sub else ""))


def golden(case):
    with open(os.path.join(GOLD, "philox_%s.json" % case)) as fh:
        return json.load(fh)


def inst_paths(name):
    d = os.path.join(INST, name)
    return os.path.join(d, "categories.csv"), os.path.join(d, "respondents.csv")


PHILOX_CASES = sorted(f[len("philox_"):-len(".json")] for f in os.listdir(GOLD)
                      if f.startswith("philox_") and f.endswith(".json"))


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    # gpu-marked tests must not silently pass without the device path
    assert torch.cuda.is_available(), "gpu test collected but no HIP device is visible"
    return True
