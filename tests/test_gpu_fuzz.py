"""Property-based differential tests (hypothesis) of every device mode against
the CPU oracle: random key sizes, lengths across the launch-shape boundaries
(256x1 up to 1 MiB, 1024x1 up to 4 MiB, persistent bulk above), byte offsets
into a larger buffer (misaligned views are staged by the Python layer), in
place and out of place, random counters and block offsets near the 2^64
carry.  SURVEY.md section 4, items 2-3."""
import os

import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from our_tree_amd import ops
from our_tree_amd.models import cpu_ref

pytestmark = pytest.mark.gpu

FUZZ = settings(max_examples=40, deadline=None, derandomize=True,
                suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])

# lengths around the tail, the 64 KiB / 1 MiB / 4 MiB launch-shape switches
LENGTHS = st.one_of(st.integers(0, 5000),
                    st.sampled_from([65535, 65536, 65537, (1 << 20) - 16, 1 << 20, (1 << 20) + 16,
                                     (4 << 20) - 16, 4 << 20, (4 << 20) + 16, (5 << 20) + 3]))


def host(t):
    return t.cpu().numpy().tobytes()


def _buf(dev, n, shift, seed):
    g = torch.Generator().manual_seed(seed)
    full = torch.randint(0, 256, (n + shift + 16,), dtype=torch.uint8, generator=g).to(dev)
    return full[shift:shift + n]


@FUZZ
@given(bits=st.sampled_from([128, 192, 256]), n=LENGTHS, shift=st.integers(0, 15), inplace=st.booleans(),
       high=st.sampled_from([0, 2**64 - 3, 2**64 - 70000, 2**128 - 2]), off=st.integers(0, 1 << 20),
       seed=st.integers(0, 2**31), impl=st.sampled_from(["auto", "bitslice"]))
def test_ctr_fuzz(gpu, bits, n, shift, inplace, high, off, seed, impl):
    key = os.urandom(bits // 8)
    ctr0 = ((high + seed) % 2**128).to_bytes(16, "big")
    x = _buf(gpu, n, shift, seed)
    src = host(x)
    y = ops.ctr(x, key, ctr0, out=x if inplace else None, block_offset=off, impl=impl)
    torch.cuda.synchronize()
    assert host(y) == cpu_ref.ctr(key, ctr0, src, block_offset=off)


@FUZZ
@given(bits=st.sampled_from([128, 192, 256]), nb=st.one_of(st.integers(0, 400),
                                                           st.sampled_from([4096, 65536, 65537, 262144, 262160])),
       shift=st.integers(0, 15), inplace=st.booleans(), seed=st.integers(0, 2**31),
       mode=st.sampled_from(["ecb", "ecb-bitslice", "ecb-dec", "cbc-dec", "cfb-dec"]))
def test_block_modes_fuzz(gpu, bits, nb, shift, inplace, seed, mode):
    key, iv = os.urandom(bits // 8), os.urandom(16)
    x = _buf(gpu, 16 * nb, shift, seed)
    src = host(x)
    out = x if inplace else None
    if mode == "ecb":
        y, exp = ops.ecb_encrypt(x, key, out=out), cpu_ref.ecb(key, src)
    elif mode == "ecb-bitslice":  # split bulk / edge launches of the bitsliced kernel
        y, exp = ops.ecb_encrypt(x, key, out=out, impl="bitslice"), cpu_ref.ecb(key, src)
    elif mode == "ecb-dec":
        y, exp = ops.ecb_decrypt(x, key, out=out), cpu_ref.ecb(key, src, decrypt=True)
    elif mode == "cbc-dec":
        y, exp = ops.cbc_decrypt(x, key, iv, out=out), cpu_ref.cbc(key, iv, src, decrypt=True)
    else:
        y, exp = ops.cfb128_decrypt(x, key, iv, out=out), cpu_ref.cfb128(key, iv, src, decrypt=True)
    torch.cuda.synchronize()
    assert host(y) == exp


@FUZZ
@given(bits=st.sampled_from([128, 256]), nseg=st.integers(1, 300), seg_blocks=st.sampled_from([1, 2, 7, 32, 256]),
       shift=st.integers(0, 15), seed=st.integers(0, 2**31))
def test_cbc_segments_fuzz(gpu, bits, nseg, seg_blocks, shift, seed):
    """sector-parallel CBC: oracle and round trip, any sector size"""
    key, iv0 = os.urandom(bits // 8), os.urandom(16)
    seg = 16 * seg_blocks
    x = _buf(gpu, seg * nseg, shift, seed)
    src = host(x)
    c = ops.cbc_encrypt_segments(x, key, iv0, seg)
    torch.cuda.synchronize()
    assert host(c) == cpu_ref.cbc_segments(key, iv0, src, seg)
    p = ops.cbc_decrypt_segments(c, key, iv0, seg)
    torch.cuda.synchronize()
    assert host(p) == src
