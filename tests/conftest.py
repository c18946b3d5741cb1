import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "styletts-zs_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built libstzs_hip.so")
    config.addinivalue_line("markers", "slow: long-running CPU oracle case")


@pytest.fixture(scope="session")
def tiny():
    from stzs.spec import SPEC_TINY
    return SPEC_TINY


@pytest.fixture(scope="session")
def tiny_params(tiny):
    from stzs.params import init_params
    return init_params(tiny, seed=0)


@pytest.fixture(scope="session")
def gpu_device():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible (run with -m 'not gpu' on CPU hosts)")
    return torch.device("cuda:0")
