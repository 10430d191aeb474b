"""Shared pytest configuration.

``-m gpu`` tests need a real MI355X (run through gpurun); ``-m "not gpu"``
tests run on the CPU-only build container: oracle vs the reference's golden
fixtures, simulators, host logic, the C-ABI library's exports, and the
multi-rank (gloo) replicate-sharding path.
"""

import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run via gpurun")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


@pytest.fixture(scope="session")
def golden_runs():
    return load_golden("pf_runs")


@pytest.fixture(scope="session")
def golden_sv():
    return load_golden("sv_data")


@pytest.fixture(scope="session")
def golden_l96():
    return load_golden("l96_data")


@pytest.fixture(scope="session")
def golden_mat():
    return load_golden("mat_data")


@pytest.fixture(scope="session")
def golden_resample():
    return load_golden("resample_idx")
