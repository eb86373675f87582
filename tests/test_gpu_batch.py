"""Batched multi-message CTR (one launch for many messages with their own keys
and counters) and HIP-graph capture of the device ops, against the C oracle."""
import os

import numpy as np
import pytest
import torch

from our_tree_amd import ops
from our_tree_amd.models import cpu_ref

pytestmark = pytest.mark.gpu


def host(t):
    return t.cpu().numpy().tobytes()


def _messages(dev, sizes, seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randint(0, 256, (n,), dtype=torch.uint8, generator=g).to(dev) for n in sizes]


@pytest.mark.parametrize("tile_blocks", [64, 128, 256])
def test_ctr_batch_matches_oracle(gpu, tile_blocks):
    """Odd lengths (tails), empty messages, mixed AES-128/192/256 keys shared
    between messages, counters at the 2^64 carry and the 2^128 wrap, every
    tile size."""
    rng = np.random.default_rng(5)
    sizes = [0, 1, 15, 16, 17, 4095, 4096, 4097, 65541, 300000] + [int(v) for v in rng.integers(0, 20000, 120)]
    keys = [os.urandom(b) for b in (16, 24, 32) for _ in range(4)]
    kidx = [int(v) for v in rng.integers(0, len(keys), len(sizes))]
    ctrs = [os.urandom(16) for _ in sizes]
    ctrs[3] = os.urandom(8) + (2**64 - 3).to_bytes(8, "big")
    ctrs[8] = b"\xff" * 16                                   # 2^128 wrap inside a counter-aligned message
    ctrs[9] = os.urandom(8) + (2**64 - 5000).to_bytes(8, "big")  # 2^64 carry inside one
    xs = _messages(gpu, sizes, 1)
    outs = ops.ctr_batch(xs, keys, ctrs, key_index=kidx, tile_blocks=tile_blocks)
    torch.cuda.synchronize()
    for i, (x, y) in enumerate(zip(xs, outs)):
        assert host(y) == cpu_ref.ctr(keys[kidx[i]], ctrs[i], host(x)), f"message {i} ({sizes[i]} bytes)"


def test_packed_batch_matches_oracle(gpu):
    """Messages packed in one buffer (default back-to-back 16-byte slots and
    explicit offsets), counters as an (n, 16) array, in place and out of place."""
    rng = np.random.default_rng(9)
    lens = [int(v) for v in rng.integers(0, 9000, 300)] + [0, 1, 4096]
    slots = [(n + 15) // 16 * 16 for n in lens]
    buf = _messages(gpu, [sum(slots)], 10)[0]
    keys = [os.urandom(16), os.urandom(32)]
    kidx = [i % 2 for i in range(len(lens))]
    ctrs = rng.integers(0, 256, (len(lens), 16), dtype=np.uint8)
    ctrs[5, 8:] = 0xFF  # 2^64 carry
    src = host(buf)
    b = ops.CtrBatch.packed(buf, lens, keys, ctrs, key_index=kidx)
    b.run()
    torch.cuda.synchronize()
    got, off = host(b.out), 0
    for i, n in enumerate(lens):
        assert got[off:off + n] == cpu_ref.ctr(keys[kidx[i]], ctrs[i].tobytes(), src[off:off + n]), f"message {i}"
        off += slots[i]
    # explicit offsets, reversed order, in place
    offs = np.cumsum([0] + slots[:-1])[::-1].copy()
    lens_r = lens[::-1]
    b2 = ops.CtrBatch.packed(buf, lens_r, keys, ctrs[::-1], out=buf, offsets=offs, key_index=kidx[::-1])
    b2.run()
    torch.cuda.synchronize()
    got = host(buf)
    for j, n in enumerate(lens_r):
        o = int(offs[j])
        assert got[o:o + n] == cpu_ref.ctr(keys[kidx[::-1][j]], ctrs[::-1][j].tobytes(), src[o:o + n])


def test_ctr_batch_in_place_replay(gpu):
    """in == out, planned once and run twice: CTR twice is the identity."""
    sizes = [4096 * 3, 1000, 8192 + 48]
    xs = _messages(gpu, sizes, 2)
    ref = [x.clone() for x in xs]
    keys = [os.urandom(16) for _ in sizes]
    ctrs = [os.urandom(16) for _ in sizes]
    b = ops.CtrBatch(xs, keys, ctrs, outs=xs)
    b.run()
    torch.cuda.synchronize()
    assert host(xs[1]) == cpu_ref.ctr(keys[1], ctrs[1], host(ref[1]))
    b.run()
    torch.cuda.synchronize()
    assert all(torch.equal(x, r) for x, r in zip(xs, ref))


def test_ops_under_hip_graph_capture(gpu):
    """ops.ctr and CtrBatch.run only enqueue kernels on the current stream (no
    allocation or synchronisation), so they can be captured into a HIP graph
    (torch.cuda.CUDAGraph) and replayed."""
    key, ctr0 = os.urandom(16), os.urandom(16)
    x = _messages(gpu, [(1 << 20) + 5], 3)[0]
    y = torch.empty_like(x)
    xs = _messages(gpu, [4096, 777, 12288], 4)
    keys = [os.urandom(32) for _ in xs]
    ctrs = [os.urandom(16) for _ in xs]
    batch = ops.CtrBatch(xs, keys, ctrs)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # warm up outside the capture
        ops.ctr(x, key, ctr0, out=y)
        batch.run()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        ops.ctr(x, key, ctr0, out=y)
        batch.run()
    y.zero_()
    for o in batch.outs:
        o.zero_()
    graph.replay()
    torch.cuda.synchronize()
    assert host(y) == cpu_ref.ctr(key, ctr0, host(x))
    for x_, o, k, c in zip(xs, batch.outs, keys, ctrs):
        assert host(o) == cpu_ref.ctr(k, c, host(x_))
