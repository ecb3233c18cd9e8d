"""Test configuration: the `gpu` marker, repo-root import path and shared fixtures.

`-m "not gpu"` tests run on the CPU container (oracle vs golden vectors, host logic, C-ABI
symbol checks, gloo multi-process sharding).  `-m gpu` tests are the parity tests proper:
they call the HIP kernels through the C ABI and compare with the oracle / golden fixtures.
"""
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests")


@pytest.fixture(scope="session")
def golden_S():
    return np.load(GOLDEN / "synthetic_S.npz", allow_pickle=False)


@pytest.fixture(scope="session")
def golden_kat():
    return np.load(GOLDEN / "dedicom_kat.npz", allow_pickle=False)


def rel_err(got, want) -> float:
    """max|got - want| / max|want| — the SURVEY §8c tolerance metric."""
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    den = np.max(np.abs(want))
    if den == 0:
        return float(np.max(np.abs(got)))
    return float(np.max(np.abs(got - want)) / den)
