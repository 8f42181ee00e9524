import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def K(dev):
    """The HIP kernel extension; must load on a GPU box (no silent fallback)."""
    from distributed_tensorflow_ibm_mnist_amd.ops._ext import kernels
    return kernels()


@pytest.fixture
def grid_cap(K):
    """Cap every persistent kernel's grid (K.set_grid_cap) for one test, so a small batch
    runs the multi-iteration paths (several tiles / images per block) that the benchmark
    batches run; reset afterwards."""
    yield K.set_grid_cap
    K.set_grid_cap(0)
