import os
import sys

import pytest

try:  # import torch before libpmhip.so is loaded: one HIP runtime per process (see pmrender/hip.py)
    import torch  # noqa: F401
except ImportError:
    pass

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-raytrace_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); runs the HIP kernels through the C-ABI")
    config.addinivalue_line("markers", "slow: larger CPU-side cases")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.load()
    return oracle


@pytest.fixture(scope="session")
def hip_mod():
    from pmrender import hip
    hip.load_library()
    return hip
