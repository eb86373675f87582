"""Monte-Carlo known-answer chains of the reference self-test
(/root/reference/aes-modes/aes.c:912-950 vectors, loop :1084-1200): 10,000
chained ECB / CBC operations from an all-zero key, block and IV at
128/192/256 bits.  The CPU oracle runs them in C (aes_self_test); the GPU test
drives the HIP ECB (T-table and bitsliced), CBC-decrypt and CBC-encrypt
(sector kernel, one 1-block segment) kernels through the same chains, on 64
identical lanes at once for ECB so every lane of a wave is checked."""
import ctypes

import pytest

from our_tree_amd import _native

MODES = {"ecb-enc": 0, "ecb-dec": 1, "cbc-enc": 2, "cbc-dec": 3}
CASES = [(m, b) for m in MODES for b in (128, 192, 256)]


def expected(mode, bits):
    return bytes.fromhex(_native.cpu_lib().aes_monte_carlo_expected(MODES[mode], bits).decode())


@pytest.mark.parametrize("mode,bits", CASES)
def test_cpu_monte_carlo(mode, bits):
    out = (ctypes.c_uint8 * 16)()
    assert _native.cpu_lib().aes_monte_carlo(MODES[mode], bits, out) == 0
    assert bytes(out) == expected(mode, bits)


@pytest.mark.gpu
@pytest.mark.parametrize("mode,bits", CASES)
def test_gpu_monte_carlo(gpu, mode, bits):
    import torch

    from our_tree_amd import ops

    key = bytes(bits // 8)
    exp = expected(mode, bits)
    if mode in ("ecb-enc", "ecb-dec"):
        impls = ("ttable", "bitslice") if mode == "ecb-enc" else (None,)
        for impl in impls:
            buf = torch.zeros(64 * 16, dtype=torch.uint8, device=gpu)
            for _ in range(10000):
                if mode == "ecb-enc":
                    ops.ecb_encrypt(buf, key, out=buf, impl=impl)
                else:
                    ops.ecb_decrypt(buf, key, out=buf)
            got = buf.view(64, 16).cpu()
            assert all(bytes(got[i].tolist()) == exp for i in range(64)), impl
    elif mode == "cbc-dec":
        buf = torch.zeros(16, dtype=torch.uint8, device=gpu)
        iv = bytes(16)
        for _ in range(10000):
            nxt = bytes(buf.cpu().tolist())  # the ciphertext block is the next IV
            ops.cbc_decrypt(buf, key, iv, out=buf)
            iv = nxt
        assert bytes(buf.cpu().tolist()) == exp
    else:
        buf = torch.zeros(16, dtype=torch.uint8, device=gpu)
        out = torch.empty_like(buf)
        prv = torch.zeros_like(buf)
        iv = bytes(16)
        for _ in range(10000):
            ops.cbc_encrypt_segments(buf, key, iv, 16, out=out)
            iv = bytes(out.cpu().tolist())
            buf.copy_(prv)
            prv.copy_(out)
        assert bytes(prv.cpu().tolist()) == exp
