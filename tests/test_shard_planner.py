"""Shard planner + "fake multi-GPU": the distribution logic (counter offsets,
CBC halos, equal-count scatter plans) verified on the CPU oracle with N logical
shards."""
import os

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from our_tree_amd.models import cpu_ref
from our_tree_amd.parallel import shard as sh


@given(st.integers(0, 10**7), st.integers(1, 64))
@settings(max_examples=200, deadline=None)
def test_plan_covers_everything(n, k):
    p = sh.plan(n, k)
    assert len(p) == k
    assert p[0].offset == 0 and p[-1].end == n
    for a, b in zip(p, p[1:]):
        assert a.end == b.offset
    for s in p[:-1]:
        assert s.nbytes % 16 == 0
    sizes = [s.nbytes for s in p[:-1]]
    if sizes:
        assert max(sizes) - min(sizes) <= 16
    assert all(s.block_offset * 16 == s.offset for s in p)


@pytest.mark.parametrize("k", [1, 2, 3, 4, 8])
def test_fake_multi_gpu_ctr(k):
    key, ctr0 = os.urandom(16), (2**64 - 17).to_bytes(16, "big")
    data = os.urandom(16 * 1001 + 9)
    ref = cpu_ref.ctr(key, ctr0, data)
    out = b"".join(cpu_ref.ctr(key, ctr0, data[s.offset:s.end], s.block_offset) for s in sh.plan(len(data), k))
    assert out == ref


@pytest.mark.parametrize("k", [1, 2, 5, 8])
def test_fake_multi_gpu_cbc_decrypt_halo(k):
    key, iv = os.urandom(32), os.urandom(16)
    pt = os.urandom(16 * 777)
    ct = cpu_ref.cbc(key, iv, pt)
    shards = sh.plan(len(ct), k)
    halos = sh.cbc_halos(ct, iv, shards)
    out = b"".join(cpu_ref.cbc(key, h, ct[s.offset:s.end], decrypt=True) for s, h in zip(shards, halos))
    assert out == pt


def test_ctr_add_wrap_modes():
    c = (2**64 - 1).to_bytes(16, "big")
    assert sh.ctr_add(c, 1) == (2**64).to_bytes(16, "big")
    assert sh.ctr_add(c, 1, wrap64=True) == bytes(16)
    assert sh.ctr_add(b"\xff" * 16, 1) == bytes(16)


def test_equal_plan():
    per, tot = sh.equal_plan(1000, 3)
    assert per % 16 == 0 and tot == 3 * per and tot >= 1000


def test_chunks():
    c = sh.chunks(1000, 100)
    assert c[0] == (0, 96) and sum(n for _, n in c) == 1000


def test_rfc3686_block():
    assert sh.rfc3686_block(b"\x00\x00\x00\x30", bytes(8)).hex() == "00000030000000000000000000000001"
