import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built libotc.so")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def gpu():
    """GPU tests must exercise the native HIP path: fail loudly (not skip) if
    the library is missing or no GPU is visible."""
    import torch

    from our_tree_amd import _native

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but torch.cuda.is_available() is False")
    _native.require_gpu_lib()
    return torch.device("cuda", 0)
