"""Allocation-failure injection on a healthy GPU ("Failure
detection / fault injection"): ``otc_fault_inject_alloc(n)`` makes the
(n+1)-th runtime allocation from now fail once -- device chunk buffers,
NUMA-pinned host windows, RCCL job buffers, the bitsliced kernel's per-call
tables.  Every entry point must then fail cleanly with an error (or, for the
bitsliced CTR tables, fall back to the uncached kernel, and for the claimed
kernels to the T-table, with identical output), release what it had built,
and work again on the next call."""
import os

import numpy as np
import pytest
import torch

from our_tree_amd import _native, ops
from our_tree_amd.models import cpu_ref
from our_tree_amd.parallel import stream as pstream

pytestmark = pytest.mark.gpu


@pytest.fixture
def inject(gpu):
    lib = _native.require_gpu_lib()
    yield lib.otc_fault_inject_alloc
    lib.otc_fault_inject_alloc(-1)


def _rnd(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)


def test_engine_create_and_run_under_alloc_faults(inject):
    key, ctr = os.urandom(16), os.urandom(16)
    x = _rnd((3 << 20) + 5, 1)
    ref = cpu_ref.ctr(key, ctr, x.tobytes())
    failed = 0
    for k in range(12):
        inject(k)
        try:
            with pstream.StreamEngine(0, chunk_bytes=1 << 20, depth=3) as eng:
                y = np.zeros_like(x)
                eng.run("ctr", x, y, key, ctr)
                assert y.tobytes() == ref  # the fault landed after this call's allocations
        except RuntimeError as e:
            failed += 1
            assert "otc_engine" in str(e)
        finally:
            inject(-1)
    assert failed >= 6  # 3 x (d_in, d_out) device buffers at least
    with pstream.StreamEngine(0, chunk_bytes=1 << 20, depth=3) as eng:
        y = np.zeros_like(x)
        eng.run("ctr", x, y, key, ctr)
    assert y.tobytes() == ref


def test_multi_rccl_job_under_alloc_faults(inject):
    key, iv = os.urandom(32), os.urandom(16)
    x = pstream.pinned_empty((2 << 20) + 48)
    x[:] = _rnd(x.nbytes, 2)
    ref = cpu_ref.cbc(key, iv, x.tobytes(), decrypt=True)
    failed = 0
    y = pstream.pinned_empty(x.nbytes)  # before arming: the injected faults are the job's own
    for k in range(8):
        y[:] = 0
        inject(k)
        try:
            pstream.multi_gpu_run("cbc-dec", x, y, key, iv, ngpus=1, strategy="rccl", chunk_bytes=256 << 10)
            assert y.tobytes() == ref
        except RuntimeError as e:
            failed += 1
            assert "otc_multi_run" in str(e)
        finally:
            inject(-1)
        _native.require_gpu_lib().otc_release_resources()  # next attempt builds the job afresh
    assert failed >= 4  # 2 x (pin, pout) + 2 x (root_in, root_out)
    y = pstream.pinned_empty(x.nbytes)
    pstream.multi_gpu_run("cbc-dec", x, y, key, iv, ngpus=1, strategy="rccl", chunk_bytes=256 << 10)
    assert y.tobytes() == ref


@pytest.mark.parametrize("bits", [128, 256])
def test_bitslice_ctr_falls_back_without_group_table(inject, gpu, bits):
    """No room for the counter-caching tables: the uncached kernel runs."""
    key, ctr = os.urandom(bits // 8), os.urandom(8) + (2**64 - 50000).to_bytes(8, "big")
    x = torch.from_numpy(_rnd(16 * 100000 + 3, 3)).to(gpu)
    inject(0)
    y = ops.ctr(x, key, ctr, impl="bitslice")
    torch.cuda.synchronize()
    assert y.cpu().numpy().tobytes() == cpu_ref.ctr(key, ctr, x.cpu().numpy().tobytes())


@pytest.mark.parametrize("k", [0, 1])
def test_bitslice_ecb_alloc_failure_falls_back(inject, gpu, k):
    """impl="bitslice" ECB is the bitsliced claim kernel alone (split_claim,
    bs_only).  If its work counter (allocation 0) or key table (allocation 1)
    cannot be allocated, the T-table runs the call instead -- complete output,
    and last_impl() says so -- and the next call runs bitsliced again."""
    key = os.urandom(16)
    x = torch.from_numpy(_rnd(16 * 4096 * 3 + 32, 4)).to(gpu)
    ref = cpu_ref.ecb(key, x.cpu().numpy().tobytes())
    inject(k)
    y = ops.ecb_encrypt(x, key, impl="bitslice")
    torch.cuda.synchronize()
    assert ops.last_impl() == "ttable"
    assert y.cpu().numpy().tobytes() == ref
    inject(-1)
    y = ops.ecb_encrypt(x, key, impl="bitslice")
    torch.cuda.synchronize()
    assert ops.last_impl() == "bitslice"
    assert y.cpu().numpy().tobytes() == ref


@pytest.mark.parametrize("k,want", [(0, "ttable"), (1, "ttable")])
def test_split_under_alloc_faults(inject, gpu, k, want):
    """The claimed split's work counter (allocation 0) or the bitsliced half's
    key table (allocation 1) cannot be allocated: the T-table runs every unit
    (plain, or as the split's only claimant) and the output is complete."""
    key, iv = os.urandom(32), os.urandom(16)
    x = torch.from_numpy(_rnd(16 * 2048 * 40 + 48, 5)).to(gpu)
    ref_ecb = cpu_ref.ecb(key, x.cpu().numpy().tobytes())
    inject(k)
    y = ops.ecb_encrypt(x, key, impl="split")
    torch.cuda.synchronize()
    assert ops.last_impl() == want
    assert y.cpu().numpy().tobytes() == ref_ecb
    inject(-1)
    inject(k)
    z = ops.cbc_decrypt(x, key, iv, impl="split")
    torch.cuda.synchronize()
    assert z.cpu().numpy().tobytes() == cpu_ref.cbc(key, iv, x.cpu().numpy().tobytes(), decrypt=True)
    inject(-1)
    y = ops.ecb_encrypt(x, key, impl="split")
    torch.cuda.synchronize()
    assert ops.last_impl() == "split" and y.cpu().numpy().tobytes() == ref_ecb
