"""The config-4 scatter/encrypt/gather job (parallel/jobs.py) verifies EVERY
rank's piece, observes the bytes that crossed between ranks, and fails when
one rank's piece is corrupted -- gloo on CPU at world sizes 2, 4 and 8 (the
same code runs over RCCL on MI355X)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, decrypt, fault, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from our_tree_amd.parallel import dist as pdist
    from our_tree_amd.parallel import jobs

    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pdist.reset_groups()
        res = jobs.cbc_scatter_job(3, 4096, b"k" * 32, bytes(range(16)), sector=512, decrypt=decrypt,
                                   device="cpu", fault=fault)
        q.put((rank, res))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


def _run(world, decrypt=False, fault=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, decrypt, fault, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r, v in res.items():
        assert isinstance(v, dict), f"rank {r} failed: {v}"
    return res


@pytest.mark.parametrize("world,decrypt", [(2, False), (4, False), (8, False), (4, True)])
def test_every_rank_verified(world, decrypt):
    res = _run(world, decrypt)
    piece = 4096 + (16 if decrypt else 0)
    for r, v in res.items():
        assert v["verified"], v
        assert v["ranks_verified"] == world and v["per_rank_ok"] == [True] * world
        assert v["collectives"] and v["backend"] == "gloo"
        # observed: every non-root piece out and back, in the warmup and last
        # round -- over gloo, i.e. host memory, never labelled xGMI
        assert v["transport"] == "host"
        assert v["peer_bytes_verified"] == v["host_bytes_verified"] == 2 * 2 * (world - 1) * piece
        assert v["peer_bytes_timed"] == v["host_bytes_timed"] == 2 * 3 * (world - 1) * piece
        assert v["xgmi_bytes_verified"] == 0 and v["xgmi_bytes_timed"] == 0


@pytest.mark.parametrize("world,where", [(4, "recv"), (8, "recv"), (4, "out")])
def test_corrupted_piece_on_rank3_fails(world, where):
    res = _run(world, fault=(3, where))
    for r, v in res.items():
        assert not v["verified"], v
        assert v["per_rank_ok"][3] is False
        assert v["ranks_verified"] == world - 1
        assert v["peer_bytes_verified"] == 2 * 2 * (world - 2) * 4096 and v["xgmi_bytes_verified"] == 0


def test_host_checksum_matches_definition():
    from our_tree_amd.parallel.jobs import checksum

    b = bytes(range(256)) * 3
    w = [int.from_bytes(b[8 * i:8 * i + 8], "little") for i in range(len(b) // 8)]
    ref = 0
    for i, x in enumerate(w):
        ref ^= (x * (0x9E3779B97F4A7C15 | 1) + 2 * i) & (2**64 - 1)
    assert checksum(torch.frombuffer(bytearray(b), dtype=torch.uint8)) == ref
    t = torch.frombuffer(bytearray(b), dtype=torch.uint8).clone()
    t[100] ^= 1
    assert checksum(t) != ref
