"""One-process-per-rank data parallelism over torch.distributed with the gloo
backend on CPU (world sizes 1, 2, 3, 4 and 8): sharded CTR, CBC-decrypt halo exchange
(ring send/recv) and root scatter/gather must equal the single-stream oracle.
The same code runs with backend nccl (= RCCL) on MI355X GPUs."""
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


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from our_tree_amd.models import cpu_ref
    from our_tree_amd.parallel import dist as pdist

    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        key, ctr0, iv = b"K" * 16, (2**64 - 100).to_bytes(16, "big"), b"I" * 16
        g = torch.Generator().manual_seed(0)
        per = 16 * 257
        full = torch.randint(0, 256, (per * world,), dtype=torch.uint8, generator=g)
        ref_ctr = cpu_ref.ctr(key, ctr0, full.numpy().tobytes())
        mine = full[rank * per:(rank + 1) * per].clone()
        pdist.sharded_ctr_(mine, key, ctr0)
        ok1 = mine.numpy().tobytes() == ref_ctr[rank * per:(rank + 1) * per]

        ct_full = cpu_ref.cbc(key, iv, full.numpy().tobytes())
        ct = torch.frombuffer(bytearray(ct_full[rank * per:(rank + 1) * per]), dtype=torch.uint8)
        pt = pdist.cbc_decrypt_sharded(ct, key, iv)
        ok2 = pt.numpy().tobytes() == full.numpy().tobytes()[rank * per:(rank + 1) * per]

        # several rounds (2 KiB per rank per round, uneven tail): the duplex
        # pipeline (gather of round r on its own communicator, overlapping the
        # scatter of round r+1, two buffer slots) and the serial one
        n = len(ref_ctr) - 5
        ok3 = True
        for overlap in (True, False):
            res = pdist.scatter_ctr(full[:n] if rank == 0 else None, n, key, ctr0, chunk_per_rank=1024,
                                    overlap=overlap)
            ok3 = ok3 and (res is None if rank != 0 else res.numpy().tobytes() == ref_ctr[:n])
        # OTC_DUPLEX=0: every pipeline falls back to the one communicator
        os.environ["OTC_DUPLEX"] = "0"
        ok3 = ok3 and not pdist.ScatterGatherPipeline(1024).overlap
        del os.environ["OTC_DUPLEX"]
        ok3 = ok3 and pdist.ScatterGatherPipeline(1024).overlap
        m = pdist.allreduce_max(float(rank))
        ok4 = m == world - 1

        # uneven shards (shard.plan: the first ranks get one extra block, the
        # last takes the partial tail): offsets from the plan and from the
        # all_gather prefix sum must both equal the single-stream keystream
        from our_tree_amd.parallel import shard as sh

        tot = 16 * (257 * world + 3) + 5
        s = sh.plan(tot, world)[rank]
        stream = torch.randint(0, 256, (tot,), dtype=torch.uint8, generator=torch.Generator().manual_seed(1))
        ok5 = True
        for gn in (tot, None):
            mine = stream[s.offset:s.end].clone()
            src = mine.numpy().tobytes()
            pdist.sharded_ctr_(mine, key, ctr0, global_nbytes=gn)
            ok5 = ok5 and mine.numpy().tobytes() == cpu_ref.ctr(key, ctr0, src, s.block_offset)
        q.put((rank, ok1, ok2, ok3, ok4, ok5))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_gloo_data_parallel(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert len(r) == 6, f"worker failed: {r}"
        assert all(r[1:]), f"rank {r[0]} mismatch: {r}"


def test_collective_timeout_bound(monkeypatch):
    """Every group the engine creates gets a bounded collective timeout
    (default 300 s, OTC_COLLECTIVE_TIMEOUT_S overrides), not torch's 30 min."""
    from datetime import timedelta

    from our_tree_amd.parallel import dist as pdist

    monkeypatch.delenv("OTC_COLLECTIVE_TIMEOUT_S", raising=False)
    assert pdist.collective_timeout() == timedelta(seconds=300)
    monkeypatch.setenv("OTC_COLLECTIVE_TIMEOUT_S", "12.5")
    assert pdist.collective_timeout() == timedelta(seconds=12.5)
