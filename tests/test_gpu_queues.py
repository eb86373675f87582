"""Hardware-queue placement in a crowded process.

HIP maps ordinary streams onto GPU_MAX_HW_QUEUES (4) pooled hardware queues
per process; packets in one queue are processed in order, so a library stream
that shares a queue with a busy torch stream waits behind its kernels.  Both
tests run in the state a bench.py rank is in -- a 1-rank RCCL group -- plus 12
torch streams that each get a spin kernel before every call.

* The pinned H2D | kernel | D2H pipeline (otc_engine, streams on queues of
  their own) must overlap: wall < 0.75 x (H2D + kernel + D2H).  On pooled
  queues the same run measured 14.7 GB/s and a ratio of 1.66
  (profiles/r6/pipeline/census.jsonl; 41.8 GB/s, 0.545 on dedicated queues).
* Every co-resident split mode must really co-run: the bitsliced half (front)
  and the T-table half (back) each take >= 5% of the claim units.  A split
  whose halves serialise still produces correct bytes -- that is how round 4's
  padded-descriptor build passed every byte test -- so only the unit count
  shows it.  Negative control: the variant build
  ``make variant NAME=padclaim VFLAGS=-DOTC_DIAG_PAD_CLAIM`` (T-table claim
  descriptors padded to 104 VGPRs, the round-4 defect) fails this test
  (profiles/r6/coresidency/).

Reference: the reference's kernels share mutable state across threads
(/root/reference/aes-gpu/Source/AES.cu:290) and nothing checks it; SURVEY.md
section 5 (race detection) asks for run-time checks of concurrency claims.
"""
import ctypes
import os
import time

import numpy as np
import pytest
import torch

from our_tree_amd.models import cpu_ref

pytestmark = pytest.mark.gpu

_SPIN = {}


def _spin_cycles(seconds):
    if "per_s" not in _SPIN:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda._sleep(5_000_000)
        torch.cuda.synchronize()
        _SPIN["per_s"] = 5_000_000 / max(time.perf_counter() - t0, 1e-6)
    return max(1, int(_SPIN["per_s"] * seconds))


@pytest.fixture
def busy_streams(gpu):
    """12 torch streams; ``busy(s)`` queues a one-wave spin kernel of ~s
    seconds on each.  Drained at teardown."""
    streams = [torch.cuda.Stream(device=gpu) for _ in range(12)]

    def busy(seconds):
        cyc = _spin_cycles(seconds)
        for s in streams:
            with torch.cuda.stream(s):
                torch.cuda._sleep(cyc)

    yield busy
    torch.cuda.synchronize()


def test_pipeline_overlaps_beside_busy_streams(gpu, rccl_world1, busy_streams):
    from our_tree_amd.parallel import stream as pstream

    t = torch.ones(1, device=gpu)
    torch.distributed.all_reduce(t)  # the group's communicator and stream exist
    n = 1000 << 20
    rng = np.random.default_rng(11)
    key = bytes(rng.integers(0, 256, 32, dtype=np.uint8).tolist())
    hin, hout = pstream.pinned_empty(n), pstream.pinned_empty(n)
    hin[:] = rng.integers(0, 256, n, dtype=np.uint8)
    ratios = []
    with pstream.StreamEngine(gpu.index, chunk_bytes=64 << 20, depth=3) as eng:
        eng.run("ecb", hin, hout, key)
        for _ in range(5):
            busy_streams(0.025)  # about one pipeline pass
            st = eng.run("ecb", hin, hout, key)
            ratios.append(st["total_ms"] / (st["h2d_ms"] + st["kernel_ms"] + st["d2h_ms"]))
    S = 1 << 16
    assert hout[:S].tobytes() == cpu_ref.ecb(key, hin[:S].tobytes())
    assert hout[n - S:].tobytes() == cpu_ref.ecb(key, hin[n - S:].tobytes())
    ratios.sort()
    assert ratios[len(ratios) // 2] < 0.75, ratios


GIB2 = 2 << 30  # the split's threshold (engine.cpp split_min)

SPLIT_CALLS = {
    "ECB-256": lambda ops, x, o, k, iv: ops.ecb_encrypt(x, k, out=o),
    "ECB-dec-256": lambda ops, x, o, k, iv: ops.ecb_decrypt(x, k, out=o),
    "CBC-dec-256": lambda ops, x, o, k, iv: ops.cbc_decrypt(x, k, iv, out=o),
    "CFB-dec-256": lambda ops, x, o, k, iv: ops.cfb128_decrypt(x, k, iv, out=o),
    "CBC-dec-seg-256": lambda ops, x, o, k, iv: ops.cbc_decrypt_segments(x, k, iv, 4096, out=o),
    "CFB-dec-seg-256": lambda ops, x, o, k, iv: ops.cfb128_decrypt_segments(x, k, iv, 4096, out=o),
}

ORACLE = {
    "ECB-256": lambda k, iv, d: cpu_ref.ecb(k, d),
    "ECB-dec-256": lambda k, iv, d: cpu_ref.ecb(k, d, decrypt=True),
    "CBC-dec-256": lambda k, iv, d: cpu_ref.cbc(k, iv, d, decrypt=True),
    "CFB-dec-256": lambda k, iv, d: cpu_ref.cfb128(k, iv, d, decrypt=True),
    "CBC-dec-seg-256": lambda k, iv, d: cpu_ref.cbc_segments(k, iv, d, 4096, decrypt=True),
    "CFB-dec-seg-256": lambda k, iv, d: cpu_ref.cfb128_segments(k, iv, d, 4096, decrypt=True),
}


@pytest.fixture(scope="module")
def split_bufs(gpu):
    from our_tree_amd import ops

    x = torch.empty(GIB2, dtype=torch.uint8, device=gpu)
    ops.fill_random_(x, seed=21)
    o = torch.empty_like(x)
    # No warm-up: the process's first split call must co-run too.  (It did
    # not before the library paid the auxiliary streams' one-time costs at
    # their creation -- the bitsliced code object, a first submission per
    # queue: front 0 in exactly the first of 64 calls of
    # profiles/r6/coresidency/matrix.jsonl, 19.7 ms against 1.9.)
    yield x, o
    del x, o


@pytest.mark.parametrize("mode", list(SPLIT_CALLS))
def test_split_halves_coresident_in_busy_process(gpu, rccl_world1, busy_streams, split_bufs, mode):
    from our_tree_amd import _native, ops

    lib = _native.require_gpu_lib()
    x, o = split_bufs
    key, iv = bytes(range(32)), bytes(range(0x40, 0x50))
    t = torch.ones(1, device=gpu)
    torch.distributed.all_reduce(t)
    fr, bk, nu = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    lib.otc_split_stats(1)
    try:
        busy_streams(0.002)
        SPLIT_CALLS[mode](ops, x, o, key, iv)
        torch.cuda.synchronize()
        ran = ops.last_impl()
        assert lib.otc_split_last_units(ctypes.byref(fr), ctypes.byref(bk), ctypes.byref(nu)) == 0
    finally:
        lib.otc_split_stats(0)
    assert ran == "split", (mode, ran, ops.split_fallback_reason())
    front, back, n = fr.value, bk.value, nu.value
    assert n > 0 and front + back == n
    # both halves took work: they ran at the same time (a serialised pair
    # leaves one side with ~0 units, profiles/r5/coresidency/)
    assert front >= 0.05 * n and back >= 0.05 * n, (mode, front, back, n)
    S = 1 << 16
    head = x[:S].cpu().numpy().tobytes()
    assert o[:S].cpu().numpy().tobytes() == ORACLE[mode](key, iv, head), mode
    if os.environ.get("OTC_PRINT_UNITS"):
        print(mode, front, back, n)


def test_split_fallback_reason(gpu):
    """A split request that cannot split runs the T-table and says why
    (otc_split_fallback_reason); one that splits leaves it empty."""
    from our_tree_amd import ops

    key = bytes(range(32))
    x = torch.empty(2048 * 16, dtype=torch.uint8, device=gpu)  # one claim unit: too few to split
    ops.fill_random_(x, seed=3)
    y = ops.ecb_encrypt(x, key, impl="split")
    torch.cuda.synchronize()
    assert ops.last_impl() == "ttable"
    assert ops.split_fallback_reason() == "too few claim units"
    assert host_bytes(y) == cpu_ref.ecb(key, host_bytes(x))
    x = torch.empty(64 * 2048 * 16, dtype=torch.uint8, device=gpu)
    ops.fill_random_(x, seed=4)
    y = ops.ecb_encrypt(x, key, impl="split")
    torch.cuda.synchronize()
    assert ops.last_impl() == "split"
    assert ops.split_fallback_reason() == ""
    assert host_bytes(y) == cpu_ref.ecb(key, host_bytes(x))


def host_bytes(t):
    return t.cpu().numpy().tobytes()


def test_split_captured_in_graph(gpu):
    """A split call captured into a HIP graph (torch.cuda.CUDAGraph: stream
    capture of the fork / join events, the claim counter's stream-ordered
    allocation and both halves' launches) replays to the right bytes; a call
    made while capturing never synchronises (engine.cpp aux_take: no warm-up
    under capture)."""
    from our_tree_amd import ops

    key = bytes(range(32))
    x = torch.empty(64 * 2048 * 16, dtype=torch.uint8, device=gpu)
    ops.fill_random_(x, seed=8)
    o = torch.empty_like(x)
    ops.ecb_encrypt(x, key, out=o, impl="split")
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ops.ecb_encrypt(x, key, out=o, impl="split")
        ran = ops.last_impl()
    assert ran == "split", (ran, ops.split_fallback_reason())
    o.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert host_bytes(o) == cpu_ref.ecb(key, host_bytes(x))
    g.replay()
    torch.cuda.synchronize()
    assert host_bytes(o) == cpu_ref.ecb(key, host_bytes(x))


@pytest.mark.parametrize("pooled", [False, True])
def test_engine_queue_modes_same_bytes(gpu, pooled):
    """Both queue arms of the pinned pipeline (dedicated, the default; pooled,
    the A/B arm) produce the oracle's bytes -- CTR across chunk boundaries
    and a tail, CBC decryption with its cross-chunk halo."""
    from our_tree_amd.parallel import stream as pstream

    n = (24 << 20) + 16 * 7 + 5
    rng = np.random.default_rng(5 + pooled)
    key, ctr = bytes(rng.integers(0, 256, 16, dtype=np.uint8).tolist()), bytes(range(16))
    hin, hout = pstream.pinned_empty(n), pstream.pinned_empty(n)
    hin[:] = rng.integers(0, 256, n, dtype=np.uint8)
    with pstream.StreamEngine(gpu.index, chunk_bytes=4 << 20, depth=3, pooled_queues=pooled) as eng:
        eng.run("ctr", hin, hout, key, ctr)
        assert hout.tobytes() == cpu_ref.ctr(key, ctr, hin.tobytes())
        m = n - n % 16
        eng.run("cbc-dec", hin[:m], hout[:m], key, ctr)
        assert hout[:m].tobytes() == cpu_ref.cbc(key, ctr, hin[:m].tobytes(), decrypt=True)
