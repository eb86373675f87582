"""Host streaming pipeline (pinned 3-stream engine), single-process multi-GPU
planner (direct ingest and RCCL scatter/gather) and the torch.distributed
helpers on one GPU: results must be byte-identical to the CPU oracle."""
import os

import numpy as np
import pytest
import torch

from our_tree_amd import _native
from our_tree_amd.models import cpu_ref
from our_tree_amd.parallel import dist as pdist
from our_tree_amd.parallel import stream as pstream

pytestmark = pytest.mark.gpu


def rnd_np(n, seed=0):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)


@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("mode", ["ctr", "ecb", "cbc-dec"])
def test_engine_matches_oracle(gpu, pinned, mode):
    n = (3 << 20) + 16 * 1000 + (5 if mode == "ctr" else 0)
    key, iv = os.urandom(32), os.urandom(16)
    if pinned:
        x = pstream.pinned_empty(n)
        x[:] = rnd_np(n, 1)
        y = pstream.pinned_empty(n)
    else:
        x, y = rnd_np(n, 1), np.zeros(n, np.uint8)
    with pstream.StreamEngine(0, chunk_bytes=1 << 20, depth=3) as eng:  # many chunks, ring wrap-around
        st = eng.run(mode, x, y, key, iv, impl="auto")
    assert st["chunks"] >= 3
    data = x.tobytes()
    if mode == "ctr":
        ref = cpu_ref.ctr(key, iv, data)
    elif mode == "ecb":
        ref = cpu_ref.ecb(key, data, threads=8)
    else:
        ref = cpu_ref.cbc(key, iv, data, decrypt=True)
    assert y.tobytes() == ref


def pinned_copy(a):
    p = pstream.pinned_empty(a.nbytes)
    p[:] = a
    return p


@pytest.mark.parametrize("strategy", ["direct", "rccl"])
@pytest.mark.parametrize("mode", ["ctr", "cbc-dec"])
def test_multi_gpu_planner(gpu, strategy, mode):
    """Pinned host buffers, as config 4/5 run them (the pageable form only
    warns: test_multi_rccl_pageable_warns)."""
    ngpus = torch.cuda.device_count()
    n = (2 << 20) + 48
    key, iv = os.urandom(16), os.urandom(16)
    x, y = pinned_copy(rnd_np(n, 2)), pstream.pinned_empty(n)
    st = pstream.multi_gpu_run(mode, x, y, key, iv, ngpus=ngpus, strategy=strategy, chunk_bytes=256 << 10)
    ref = cpu_ref.ctr(key, iv, x.tobytes()) if mode == "ctr" else cpu_ref.cbc(key, iv, x.tobytes(), decrypt=True)
    assert y.tobytes() == ref
    assert st["ngpus"] == ngpus


def test_scatter_apply_gather_single_rank(gpu):
    key, ctr0 = os.urandom(16), os.urandom(16)
    n = 10_000_003
    full = torch.randint(0, 256, (n,), dtype=torch.uint8, device=gpu)
    out = pdist.scatter_ctr(full, n, key, ctr0, chunk_per_rank=1 << 20)
    assert out.cpu().numpy().tobytes() == cpu_ref.ctr(key, ctr0, full.cpu().numpy().tobytes())


def test_models_api_on_gpu(gpu):
    from our_tree_amd.models import AES, ARC4, RC4MultiStream

    key = os.urandom(24)
    aes = AES(key)
    x = torch.randint(0, 256, (16 * 999,), dtype=torch.uint8, device=gpu)
    assert torch.equal(aes.decrypt(aes.encrypt(x)), x)
    iv = os.urandom(16)
    c = aes.cbc_encrypt(x, iv, segment_bytes=16 * 37)
    assert torch.equal(aes.cbc_decrypt(c, iv, segment_bytes=16 * 37), x)
    assert c.cpu().numpy().tobytes() == aes.cbc_encrypt(x.cpu().numpy().tobytes(), iv, segment_bytes=16 * 37)
    assert torch.equal(aes.ctr(aes.ctr(x, iv), iv), x)
    a4 = ARC4(b"secret")
    y = a4.crypt(x)
    assert y.cpu().numpy().tobytes() == cpu_ref.arc4_crypt(x.cpu().numpy().tobytes(),
                                                            cpu_ref.arc4_keystream(b"secret", x.numel()))
    keys = torch.randint(0, 256, (128, 16), dtype=torch.uint8, device=gpu)
    m = RC4MultiStream(keys)
    z = torch.randint(0, 256, (128, 100), dtype=torch.uint8, device=gpu)
    assert torch.equal(m.crypt(m.crypt(z)), z)


@pytest.mark.parametrize("mode", ["ctr", "cbc-dec"])
def test_resumable_file_job_on_gpu(gpu, tmp_path, mode):
    """Interrupted + resumed file job through the pinned GPU pipeline equals
    the oracle (our_tree_amd/parallel/filejob.py)."""
    from our_tree_amd.parallel import filejob

    n = (3 << 20) + (16 if mode == "cbc-dec" else 5)
    data = os.urandom(n)
    src, dst = tmp_path / "in", tmp_path / "out"
    src.write_bytes(data)
    key, iv = os.urandom(16), os.urandom(16)
    be = filejob.gpu_backend(chunk_bytes=1 << 20)
    try:
        r = filejob.crypt_file(str(src), str(dst), key, iv, mode=mode, chunk_bytes=1 << 20, backend=be, max_chunks=1)
        assert not r["done"]
        r = filejob.crypt_file(str(src), str(dst), key, iv, mode=mode, chunk_bytes=1 << 20, backend=be)
        assert r["done"] and r["resumed_from"] == 1
    finally:
        be.close()
    ref = cpu_ref.ctr(key, iv, data) if mode == "ctr" else cpu_ref.cbc(key, iv, data, decrypt=True)
    assert dst.read_bytes() == ref


def test_cpp_blockcipher_interface(gpu):
    """csrc/include/otc_cipher.hpp (otc::BlockCipher / otc::AesGpu) through
    bin/bc_test: FIPS-197 vectors on device and host buffers, CTR/CBC host
    path == device path, error paths."""
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bin", "bc_test")
    if not os.path.exists(exe):
        pytest.fail("bin/bc_test not built (make)")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "bc_test: OK" in r.stdout, r.stdout + r.stderr


def test_cli_gpu_selftest_and_file_job(gpu, tmp_path):
    """`python -m our_tree_amd` (in process): GPU known-answer vectors and a
    resumable file job through the pinned GPU pipeline, CTR twice = identity."""
    from our_tree_amd.__main__ import main

    assert main(["selftest", "--gpu"]) == 0
    src, mid, back = tmp_path / "a.bin", tmp_path / "b.bin", tmp_path / "c.bin"
    data = os.urandom(300_007)
    src.write_bytes(data)
    for s, d in ((src, mid), (mid, back)):
        assert main(["crypt", str(s), str(d), "--key", "22" * 16, "--iv", "ff" * 16, "--chunk", "64K"]) == 0
    assert mid.read_bytes() == cpu_ref.ctr(b"\x22" * 16, b"\xff" * 16, data)
    assert back.read_bytes() == data


@pytest.mark.parametrize("pinned", [False, True])
def test_engine_cbc_dec_in_place(gpu, pinned):
    """host_in == host_out over many chunks: every chunk's halo (previous
    ciphertext block) is captured before any D2H can overwrite it."""
    n = (3 << 20) + 16 * 77
    key, iv = os.urandom(16), os.urandom(16)
    data = rnd_np(n, 5)
    if pinned:
        x = pstream.pinned_empty(n)
        x[:] = data
    else:
        x = data.copy()
    with pstream.StreamEngine(0, chunk_bytes=256 << 10, depth=3) as eng:
        eng.run("cbc-dec", x, x, key, iv)
    assert x.tobytes() == cpu_ref.cbc(key, iv, data.tobytes(), decrypt=True)


def test_engine_stats_breakdown_and_numa(gpu):
    """otc_stream_stats: kernel / H2D / D2H / host staging times from events,
    and the pinned ring placed on the GPU's NUMA node."""
    from our_tree_amd import _native

    lib = _native.require_gpu_lib()
    n = 8 << 20
    x, y = rnd_np(n, 6), np.zeros(n, np.uint8)
    key, ctr = os.urandom(16), os.urandom(16)
    with pstream.StreamEngine(0, chunk_bytes=1 << 20, depth=3) as eng:
        st = eng.run("ctr", x, y, key, ctr)
        assert y.tobytes() == cpu_ref.ctr(key, ctr, x.tobytes())
        assert st["kernel_ms"] > 0 and st["h2d_ms"] > 0 and st["d2h_ms"] > 0 and st["host_stage_ms"] > 0
        assert st["h2d_gbps"] > 1 and st["d2h_gbps"] > 1
        node = eng.numa_node
        assert node == lib.otc_device_numa_node(0) == st["numa_node"]
        if node >= 0:
            assert lib.otc_numa_node_of_addr(eng.staging_ptr(0)) == node


@pytest.mark.parametrize("nshards", [2, 4, 8])
@pytest.mark.parametrize("mode", ["ctr", "cbc-dec"])
def test_multi_direct_logical_shards(gpu, nshards, mode, monkeypatch):
    """otc_multi_run(direct) with N logical shards mapped onto the visible
    GPU(s) (OTC_SHARE_GPUS=1): N host threads, N engines, in place for CBC."""
    monkeypatch.setenv("OTC_SHARE_GPUS", "1")
    n = (1 << 20) * 3 + 16 * 13 + (7 if mode == "ctr" else 0)
    key, iv = os.urandom(32), os.urandom(16)
    x = rnd_np(n, 7 + nshards)
    ref = cpu_ref.ctr(key, iv, x.tobytes()) if mode == "ctr" else cpu_ref.cbc(key, iv, x.tobytes(), decrypt=True)
    y = x.copy() if mode == "cbc-dec" else np.zeros(n, np.uint8)
    src = y if mode == "cbc-dec" else x
    st = pstream.multi_gpu_run(mode, src, y, key, iv, ngpus=nshards, strategy="direct", chunk_bytes=256 << 10)
    assert y.tobytes() == ref
    assert st["ngpus"] == nshards and st["numa_nodes_used"] >= 0


def test_multi_direct_refuses_oversubscription_without_share(gpu, monkeypatch):
    monkeypatch.delenv("OTC_SHARE_GPUS", raising=False)
    n = 1 << 16
    x, y = rnd_np(n, 8), np.zeros(n, np.uint8)
    with pytest.raises(RuntimeError, match="ngpus out of range"):
        pstream.multi_gpu_run("ctr", x, y, os.urandom(16), os.urandom(16), ngpus=torch.cuda.device_count() + 1)


def test_multi_rccl_cbc_dec_in_place_many_rounds(gpu):
    """RCCL scatter/gather job, double-buffered pieces, in-place CBC-dec across
    >2 rounds (buffer reuse two rounds later ordered by events)."""
    ngpus = torch.cuda.device_count()
    n = (5 << 20) + 16 * 3
    key, iv = os.urandom(16), os.urandom(16)
    data = rnd_np(n, 9)
    x = pinned_copy(data)
    pstream.multi_gpu_run("cbc-dec", x, x, key, iv, ngpus=ngpus, strategy="rccl", chunk_bytes=512 << 10)
    assert x.tobytes() == cpu_ref.cbc(key, iv, data.tobytes(), decrypt=True)


def test_multi_rccl_pageable_warns(gpu):
    """The one intended pageable case: the job still equals the oracle, and
    says that its root copies will block."""
    n = (1 << 20) + 16
    key, iv = os.urandom(16), os.urandom(16)
    x, y = rnd_np(n, 10), np.zeros(n, np.uint8)
    with pytest.warns(RuntimeWarning, match="pageable"):
        pstream.multi_gpu_run("ctr", x, y, key, iv, ngpus=1, strategy="rccl", chunk_bytes=256 << 10)
    assert y.tobytes() == cpu_ref.ctr(key, iv, x.tobytes())


def test_pinned_buffers_are_seen_as_pinned(gpu):
    """pinned_empty() memory classifies as pinned, numpy memory as pageable,
    a CUDA tensor as device (otc_ptr_kind through a pointer-typed ctypes
    signature; undeclared, the address was truncated to 32 bits)."""
    p, h = pstream.pinned_empty(1 << 20), np.zeros(1 << 20, np.uint8)
    assert pstream.pageable_buffers(p, h) == [1]
    lib = _native.require_gpu_lib()
    d = torch.empty(1 << 20, dtype=torch.uint8, device=gpu)
    assert lib.otc_ptr_kind(p.ctypes.data) == pstream.PTR_PINNED
    assert lib.otc_ptr_kind(d.data_ptr()) == pstream.PTR_DEVICE


def test_engine_overlaps_h2d_cipher_d2h(gpu):
    """A 512 MiB pinned job through the 3-stream engine: H2D of chunk k+1,
    the cipher of chunk k and D2H of chunk k-1 run at once, so the wall time
    is well under the sum of the three phases' event times (SURVEY 2.4 P7;
    the reference's copies were synchronous and pageable,
    /root/reference/aes-gpu/Source/AES.cu:236,252)."""
    n = 512 << 20
    key, ctr = os.urandom(16), os.urandom(16)
    x = pstream.pinned_empty(n)
    x[: 1 << 20] = rnd_np(1 << 20, 12)
    x[1 << 20:] = 0x5A
    y = pstream.pinned_empty(n)
    with pstream.StreamEngine(0, chunk_bytes=32 << 20, depth=3) as eng:
        eng.run("ctr", x, y, key, ctr)  # warm: streams, ring, clocks
        st = eng.run("ctr", x, y, key, ctr)
    phases = st["kernel_ms"] + st["h2d_ms"] + st["d2h_ms"]
    assert st["chunks"] == 16
    assert st["total_ms"] < 0.75 * phases, st
    assert st["host_stage_ms"] == 0  # pinned: no staging copies
    assert y[: 1 << 20].tobytes() == cpu_ref.ctr(key, ctr, x[: 1 << 20].tobytes())
    tail = n - (1 << 16)
    assert y[tail:].tobytes() == cpu_ref.ctr(key, ctr, x[tail:].tobytes(), block_offset=tail // 16)


def test_multi_ctr_resident(gpu):
    ngpus = torch.cuda.device_count()
    key, ctr = os.urandom(16), (2**64 - 3).to_bytes(16, "big")
    per = 16 * 4099
    bufs = [torch.randint(0, 256, (per,), dtype=torch.uint8, device=f"cuda:{g}") for g in range(ngpus)]
    src = b"".join(b.cpu().numpy().tobytes() for b in bufs)
    ms = pstream.multi_ctr_resident(bufs, key, ctr)
    assert ms > 0
    got = b"".join(b.cpu().numpy().tobytes() for b in bufs)
    assert got == cpu_ref.ctr(key, ctr, src)


def test_multi_ctr_resident_non_byte_dtype(gpu):
    """shards of int32 / float32 are byte buffers: every byte is encrypted and
    shard g starts at counter offset g * bytes / 16 (numel was
    passed as the byte count)"""
    ngpus = torch.cuda.device_count()
    key, ctr = os.urandom(16), (2**64 - 7).to_bytes(16, "big")
    for dt in (torch.int32, torch.float32):
        per = 4 * 4099  # elements: 16 * 4099 bytes
        bufs = [torch.randint(0, 2**20, (per,), dtype=torch.int32, device=f"cuda:{g}").view(dt) for g in range(ngpus)]
        src = b"".join(b.cpu().view(torch.uint8).numpy().tobytes() for b in bufs)
        pstream.multi_ctr_resident(bufs, key, ctr)
        got = b"".join(b.cpu().view(torch.uint8).numpy().tobytes() for b in bufs)
        assert got == cpu_ref.ctr(key, ctr, src)


def test_multi_ctr_resident_rejects_bad_shards(gpu):
    key, ctr = os.urandom(16), bytes(16)
    with pytest.raises(ValueError, match="multiple of 16"):
        pstream.multi_ctr_resident([torch.zeros(20, dtype=torch.uint8, device="cuda:0")], key, ctr)
    with pytest.raises(ValueError, match="contiguous"):
        pstream.multi_ctr_resident([torch.zeros(64, dtype=torch.uint8, device="cuda:0")[::2]], key, ctr)
    with pytest.raises(ValueError, match="impl"):
        pstream.multi_ctr_resident([torch.zeros(64, dtype=torch.uint8, device="cuda:0")], key, ctr, impl="hybrid")
