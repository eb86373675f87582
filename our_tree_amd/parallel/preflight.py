"""Bounded first-contact check of the process group, before any large
allocation or timed work.

A multi-GPU run meets RCCL's peer-to-peer / IPC transport for the first time
in its first collective.  If that transport is broken (dmabuf IPC refused,
an xGMI peer missing) the collective does not fail, it hangs -- until the
launcher's 30-minute limit, with nothing in the record.  ``run`` moves 16 MiB
through the same two collectives the bench uses (scatter from the root, then
all_gather of what every rank received), checks every byte against a pattern
each rank can regenerate, and is bounded by a watchdog: if the collectives
have not finished after ``timeout_s`` the callback runs (bench.py: one error
JSON line, exit code 3), and the launcher stops the other ranks.

Result (identical on every rank): ``ok``, ``per_rank_ok`` (rank g's piece
arrived intact at g by scatter AND at every rank by all_gather), ``seconds``,
``backend``.  ``fault_rank`` flips one byte of that rank's received piece
(transport fault), ``hang_rank`` makes that rank sleep instead of joining
(hang); both are test hooks (tests/test_preflight_cpu.py, gloo at world
2/4/8).  The reference had no multi-device code.
"""
from __future__ import annotations

import os
import sys
import threading
import time

import torch
import torch.distributed as dist

from . import dist as pdist


def _pattern(n: int, rank: int, device) -> torch.Tensor:
    """Piece of rank g: bytes (31 * i + 7 * g + 1) mod 251 -- distinct per rank
    and position, reproducible anywhere without communication."""
    i = torch.arange(n, dtype=torch.int64, device=device)
    return ((31 * i + 7 * rank + 1) % 251).to(torch.uint8)


def _default_timeout(rank: int, timeout_s: float):
    print(f"preflight: rank {rank}: collectives did not finish within {timeout_s:.0f} s", file=sys.stderr,
          flush=True)
    os._exit(3)


def run(nbytes: int = 16 << 20, timeout_s: float = 120.0, on_timeout=None, fault_rank: int | None = None,
        hang_rank: int | None = None) -> dict:
    rank, world = pdist._world()
    if not pdist._pg_on():
        return {"ok": True, "per_rank_ok": [True], "seconds": 0.0, "backend": "none", "bytes": 0}
    on_timeout = on_timeout or _default_timeout
    timer = threading.Timer(timeout_s, on_timeout, args=(rank, timeout_s))
    timer.daemon = True
    timer.start()
    t0 = time.perf_counter()
    try:
        dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
        piece = max(16, (nbytes // world) // 16 * 16)
        if hang_rank == rank:
            time.sleep(timeout_s * 10)
        send = None
        if rank == 0:
            send = [_pattern(piece, g, dev) for g in range(world)]
        recv = torch.empty(piece, dtype=torch.uint8, device=dev)
        dist.scatter(recv, send, src=0)
        mine = _pattern(piece, rank, dev)
        scatter_ok = bool(torch.equal(recv, mine))
        if fault_rank == rank:
            recv[piece // 2] ^= 0x5A
        got = [torch.empty_like(recv) for _ in range(world)]
        dist.all_gather(got, recv)
        gather_ok = [bool(torch.equal(got[g], _pattern(piece, g, dev))) for g in range(world)]
        # verdict matrix: row r = what rank r saw (its scatter check + every gathered piece)
        row = torch.tensor([1 if scatter_ok else 0] + [1 if v else 0 for v in gather_ok], dtype=torch.int64,
                           device=dev)
        rows = [torch.empty_like(row) for _ in range(world)]
        dist.all_gather(rows, row)
        m = [r_.cpu().tolist() for r_ in rows]
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
    finally:
        timer.cancel()
    per_rank = [bool(m[g][0]) and all(m[r][1 + g] for r in range(world)) for g in range(world)]
    return {"ok": all(per_rank), "per_rank_ok": per_rank, "seconds": round(time.perf_counter() - t0, 3),
            "backend": dist.get_backend(), "bytes": piece * world}
