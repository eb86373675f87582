"""Host streaming pipeline (pinned 3-stream engine), single-process multi-GPU
planner (direct ingest and RCCL scatter/gather) and the torch.distributed
helpers on one GPU: results must be byte-identical to the CPU oracle."""
import os

import numpy as np
import pytest
import torch

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


@pytest.mark.parametrize("strategy", ["direct", "rccl"])
@pytest.mark.parametrize("mode", ["ctr", "cbc-dec"])
def test_multi_gpu_planner(gpu, strategy, mode):
    ngpus = torch.cuda.device_count()
    n = (2 << 20) + 48
    key, iv = os.urandom(16), os.urandom(16)
    x, y = rnd_np(n, 2), np.zeros(n, np.uint8)
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
