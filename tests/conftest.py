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


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def rccl_world1(gpu):
    """A world-size-1 RCCL (backend "nccl") process group in this process,
    torn down after the test: the same collective code path as N ranks, and
    the same streams / communicators a bench.py rank holds."""
    import torch.distributed as dist

    from our_tree_amd.parallel import dist as pdist

    if dist.is_initialized():
        pytest.skip("a process group already exists in this process")
    store = dist.TCPStore("127.0.0.1", _free_port(), 1, is_master=True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=gpu)
    pdist.reset_groups()
    try:
        yield pdist
    finally:
        dist.destroy_process_group()
        pdist.reset_groups()
