"""Shared test setup.

-m "not gpu": oracle vs golden vectors / known answers, host logic, the C-ABI
library's symbol table, gloo multi-process sharding.  -m gpu: parity of the
HIP path (through libhbx.so) against the oracle."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "binary-hologram-reinforcement-learning_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and libhbx.so")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
