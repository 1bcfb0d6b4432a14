import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "element-crush-gym_amd")
for p in (ROOT, os.path.join(ROOT, "oracle"), PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
SHAPES = {"9x9x6": (9, 9, 6), "16x16x8": (16, 16, 8)}


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running test")


def gpu_available() -> bool:
    try:
        from match3tile import _native
        return _native.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    return load
