"""Shared pytest configuration.

`gpu` marks tests that need a real MI355X (the driver runs `-m gpu` on the GPU
box and `-m "not gpu"` here, on a CPU-only container).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
DATA = os.path.join(GOLDEN, "data")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")


def data(name):
    return os.path.join(DATA, name)


@pytest.fixture
def tmpfile(tmp_path):
    def make(name):
        return str(tmp_path / name)
    return make
