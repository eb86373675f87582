"""Resumable device CTR (otc_aes_ctr_stream / ops.CtrStream) with PolarSSL
aes_crypt_ctr semantics (reference aes-modes/aes.c:869-900): one stream split
at random byte offsets over many calls equals one-shot ops.ctr AND the
byte-granular C oracle (cpu_ref.ctr_stream), with the context (nonce_counter,
stream_block, nc_off) identical to the oracle's after every call."""
import os
import random

import pytest
import torch

from our_tree_amd import ops
from our_tree_amd.models import cpu_ref

pytestmark = pytest.mark.gpu


def host(t):
    return t.cpu().numpy().tobytes()


@pytest.mark.parametrize("bits", [128, 192, 256])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_random_splits_match_one_shot_and_oracle(gpu, bits, seed):
    rng = random.Random(seed * 7 + bits)
    key = os.urandom(bits // 8)
    ctr0 = (2**64 - 37).to_bytes(16, "big") if seed == 1 else os.urandom(16)  # carry into the high half
    n = 300_000 + rng.randrange(5000)
    base = torch.randint(0, 256, (n + 64,), dtype=torch.uint8, device=gpu)
    x = base[7:7 + n]  # the stream itself starts misaligned
    one_shot = host(ops.ctr(x.clone(), key, ctr0))
    # oracle state
    nc, sb, off = bytearray(ctr0), bytearray(16), [0]
    s = ops.CtrStream(key, ctr0)
    out = torch.empty_like(x)
    pos = 0
    while pos < n:
        step = rng.choice([1, 3, 15, 16, 17, 31, 4096, 10_000, 65_537])
        step = min(step, n - pos)
        s.update(x[pos:pos + step], out=out[pos:pos + step])
        exp = cpu_ref.ctr_stream(key, nc, sb, off, host(x[pos:pos + step]))
        assert s.nc_off == off[0] and s.nonce_counter == bytes(nc)
        if off[0]:
            assert s.stream_block == bytes(sb)
        got = host(out[pos:pos + step])
        assert got == exp, (pos, step)
        pos += step
    assert host(out) == one_shot


def test_in_place_and_staged_alignments(gpu):
    """in place at every misalignment; out with a different alignment than x
    (staged by ops.CtrStream)."""
    key, ctr0 = os.urandom(16), os.urandom(16)
    n = 100_003
    src = torch.randint(0, 256, (n + 32,), dtype=torch.uint8, device=gpu)
    for a in range(16):
        x = src[a:a + n].clone() if a == 0 else src.clone()[a:a + n]
        ref = cpu_ref.ctr(key, ctr0, host(x))
        s = ops.CtrStream(key, ctr0)
        s.update(x[:5], out=x[:5])
        s.update(x[5:], out=x[5:])
        assert host(x) == ref, a
    y = torch.empty(n + 32, dtype=torch.uint8, device=gpu)
    x = src[3:3 + n]
    s = ops.CtrStream(key, ctr0)
    s.update(x[:10], out=y[1:11])
    s.update(x[10:], out=y[11:1 + n])
    assert host(y[1:1 + n]) == cpu_ref.ctr(key, ctr0, host(x))


def test_checkpoint_resume(gpu):
    """state() -> from_state() resumes mid-block exactly."""
    key, ctr0 = os.urandom(32), os.urandom(16)
    x = torch.randint(0, 256, (50_001,), dtype=torch.uint8, device=gpu)
    a = ops.CtrStream(key, ctr0)
    y1 = a.update(x[:12_345])
    b = ops.CtrStream.from_state(key, a.state())
    y2 = b.update(x[12_345:])
    assert host(y1) + host(y2) == cpu_ref.ctr(key, ctr0, host(x))
