"""Bounded RCCL first-contact check (parallel/preflight.py) and the per-rank
statistics gather bench.py reports, on gloo at world sizes 2, 4 and 8: a
clean run verifies every rank, a corrupted piece on rank 5 fails exactly that
rank everywhere, and a rank that never joins trips the watchdog instead of
hanging (round-3 review, next-round item 3)."""
import math
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, kw, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from our_tree_amd.parallel import dist as pdist
    from our_tree_amd.parallel import preflight

    def on_timeout(r, t):
        q.put((r, "timeout"))
        q.close()
        q.join_thread()  # flush the queue's feeder before the hard exit
        os._exit(3)

    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        res = preflight.run(nbytes=1 << 20, on_timeout=on_timeout, **kw)
        stats = pdist.gather_floats([rank * 10.0, float("nan") if rank == 1 else 1.5])
        q.put((rank, {"res": res, "stats": stats}))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


def _run(world, **kw):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kw, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, v = q.get(timeout=180)
            out[r] = v
            if v == "timeout":
                break
    finally:
        for p in procs:
            p.join(timeout=5)
            if p.is_alive():
                p.kill()
                p.join()
    return out


@pytest.mark.parametrize("world", [2, 4, 8])
def test_preflight_clean(world):
    out = _run(world)
    assert len(out) == world
    for r, v in out.items():
        assert isinstance(v, dict), v
        assert v["res"]["ok"] and v["res"]["per_rank_ok"] == [True] * world
        assert v["res"]["backend"] == "gloo" and v["res"]["bytes"] > 0
        rows = v["stats"]
        assert [row[0] for row in rows] == [10.0 * g for g in range(world)]
        assert math.isnan(rows[1][1]) and rows[0][1] == 1.5


@pytest.mark.parametrize("world", [8])
def test_preflight_fault_on_rank5(world):
    out = _run(world, fault_rank=5)
    for r, v in out.items():
        assert isinstance(v, dict), v
        assert not v["res"]["ok"]
        assert v["res"]["per_rank_ok"] == [g != 5 for g in range(world)]


def test_preflight_hang_trips_watchdog():
    """rank 1 never joins: the others must give up after the bound, not hang"""
    out = _run(4, hang_rank=1, timeout_s=4.0)
    assert "timeout" in out.values()
