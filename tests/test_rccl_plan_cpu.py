"""The round plan of the single-process RCCL job (otc_multi_run strategy 1,
csrc/cpu/rccl_plan.c, used by csrc/hip/pipeline.cpp rccl_job_run) at N = 2..8
on the CPU.  RCCL will not put two ranks on one GPU, so on hardware this job
has only ever run with one GPU; here its per-round pieces, CTR block offsets,
CBC-decryption halo slots and last-round padding are checked for every N and
for uneven sizes, sizes under one round and pieces of one block, and the plan
is executed with the C oracle piece by piece: the result must equal the
single-stream CTR / ECB / CBC decryption (the reference chunked per thread and
dropped the remainder, /root/reference/test.c:44-58)."""
import ctypes
import os
import random

import pytest

from our_tree_amd import _native
from our_tree_amd.models import cpu_ref
from our_tree_amd.parallel import shard as sh


def lib():
    return _native.cpu_lib()


def plan(nbytes, ngpus, piece):
    L = lib()
    nr = L.otc_rccl_nrounds(nbytes, ngpus, piece)
    out = []
    for r in range(nr):
        for g in range(ngpus):
            p = _native.RcclPiece()
            assert L.otc_rccl_plan_piece(nbytes, ngpus, piece, r, g, ctypes.byref(p)) == 0
            out.append((r, g, p))
    return nr, out


SIZES = [16, 48, 4096, 4096 * 7 + 48, 65536 * 3 + 16 * 5, 1 << 20, (1 << 20) + 16]


@pytest.mark.parametrize("ngpus", range(1, 9))
def test_pieces_partition_the_stream(ngpus):
    for nbytes in SIZES:
        for piece in (16, 64, 4096, 65536):
            nr, pcs = plan(nbytes, ngpus, piece)
            assert nr == -(-nbytes // (piece * ngpus))
            covered, end_seen = 0, False
            for r, g, p in pcs:
                assert p.round_off == r * piece * ngpus
                assert p.round_bytes + p.pad_bytes == piece * ngpus
                assert p.round_bytes == min(piece * ngpus, nbytes - p.round_off)
                assert (p.pad_bytes > 0) == (r == nr - 1 and nbytes % (piece * ngpus) != 0)
                if p.bytes == 0:
                    end_seen = True  # empty pieces only past the end
                    assert p.off == nbytes and p.halo == -1
                    continue
                assert not end_seen
                assert p.off == covered and p.off == p.round_off + g * piece
                assert p.bytes == min(piece, nbytes - p.off)
                assert p.blk0 == p.off // 16
                if p.off == 0:
                    assert p.halo == -1
                else:
                    assert p.halo == r * ngpus + g
                    assert lib().otc_rccl_halo_start(nbytes, piece, p.halo) == p.off
                covered += p.bytes
            assert covered == nbytes


def test_single_round_equals_python_equal_plan():
    """With the piece size shard.equal_plan picks for one round, the C plan's
    pieces are the Python planner's equal-count shards."""
    for ngpus in range(2, 9):
        for nbytes in (16 * 3, 4096 * 5 + 16, 1 << 20):
            per, padded = sh.equal_plan(nbytes, ngpus)
            nr, pcs = plan(nbytes, ngpus, per)
            assert nr == 1 and pcs[0][2].pad_bytes == padded - nbytes
            off = 0
            for _, g, p in pcs:
                assert p.off == min(g * per, nbytes) and p.bytes == max(0, min(per, nbytes - g * per))
                off += p.bytes
            assert off == nbytes


def test_bad_arguments():
    L = lib()
    p = _native.RcclPiece()
    assert L.otc_rccl_plan_piece(4096, 0, 64, 0, 0, ctypes.byref(p)) != 0
    assert L.otc_rccl_plan_piece(4096, 2, 0, 0, 0, ctypes.byref(p)) != 0
    assert L.otc_rccl_plan_piece(4096, 2, 64, 0, 2, ctypes.byref(p)) != 0
    assert L.otc_rccl_plan_piece(4096, 2, 64, 32, 0, ctypes.byref(p)) != 0  # round 32 of 32
    assert L.otc_rccl_nrounds(0, 4, 64) == 0


@pytest.mark.parametrize("ngpus", [2, 3, 5, 8])
def test_plan_executed_with_the_oracle(ngpus):
    """Every piece run on its own with the oracle, the way rccl_job_run runs
    it on its GPU (CTR from blk0, CBC decryption from its halo slot or the
    IV, ECB), reassembles the single-stream result."""
    rnd = random.Random(ngpus)
    key, iv = os.urandom(32), os.urandom(16)
    for nbytes, piece in ((4096 * 9 + 16 * 3, 4096), (16 * 5, 16 * 2), (16 * 40, 16 * 64), (65536 + 4096, 8192)):
        data = bytes(rnd.getrandbits(8) for _ in range(nbytes))
        nr, pcs = plan(nbytes, ngpus, piece)
        halo = lambda i: data[lib().otc_rccl_halo_start(nbytes, piece, i) - 16:][:16]
        ctr = ecb = cbc = b""
        for _, _, p in pcs:
            chunk = data[p.off:p.off + p.bytes]
            if not p.bytes:
                continue
            ctr += cpu_ref.ctr(key, iv, chunk, block_offset=p.blk0)
            ecb += cpu_ref.ecb(key, chunk)
            cbc += cpu_ref.cbc(key, iv if p.halo < 0 else halo(p.halo), chunk, decrypt=True)
        assert ctr == cpu_ref.ctr(key, iv, data), (ngpus, nbytes, piece)
        assert ecb == cpu_ref.ecb(key, data)
        assert cbc == cpu_ref.cbc(key, iv, data, decrypt=True)
