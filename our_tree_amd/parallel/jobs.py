"""Multi-rank cipher jobs shared by ``bench.py`` and ``benchmarks/``.

``cbc_scatter_job`` is BASELINE config 4 in miniature: an AES-256-CBC stream
resident on the root GPU is dealt to every rank by RCCL scatter over xGMI,
encrypted there, and gathered back (``dist.ScatterGatherPipeline``: the gather
of round r overlaps the scatter of round r+1 on a second communicator).

CBC encryption is a serial chain (/root/reference/aes-modes/aes.c:801-812),
so the parallel form encrypts independent sectors, each with the IV
``iv0 + global sector index``.  With ``decrypt`` the
job is exact single-stream CBC decryption instead: every piece carries the
16-byte ciphertext block in front of it (the halo).
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist

from ..models import cpu_ref
from . import dist as pdist
from . import shard as sh


def cbc_scatter_job(rounds: int, chunk: int, key: bytes, iv0: bytes, sector: int = 4096, decrypt: bool = False,
                    overlap: bool = True, device=None) -> dict:
    """Run 1 verified warmup round + ``rounds`` timed rounds; every rank gets
    ``chunk`` bytes per round.  Returns (on every rank) a dict with the timing,
    the verification verdict and what the communicator saw."""
    rank, world = pdist._world()
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    H = 16 if decrypt else 0
    piece_bytes = chunk + H
    pipe = pdist.ScatterGatherPipeline(piece_bytes, root=0, device=device, overlap=overlap)
    carry = torch.tensor(list(iv0), dtype=torch.uint8, device=device)
    from .. import ops

    def produce(send, r):
        if not decrypt:
            ops.fill_random_(send, seed=r)
            return
        v = send.view(world, piece_bytes)
        for g in range(world):  # synthetic ciphertext, piece by piece (rows are strided)
            ops.fill_random_(v[g, H:], seed=r * world + g)
        v[0, :H].copy_(carry)
        v[1:, :H].copy_(v[:-1, -H:])
        carry.copy_(v[-1, -H:])

    def work(piece, out, r):
        if not decrypt:
            gofs = (r * world + rank) * chunk
            ops.cbc_encrypt_segments(piece, key, sh.ctr_add(iv0, gofs // sector), sector, out=out)
            return
        # IV 0, then XOR the halo into the first block: no host round trip
        ops.cbc_decrypt(piece[H:], key, bytes(16), out=out[H:])
        out[H:2 * H].bitwise_xor_(piece[:H])

    verdict = {}

    def verify(gathered, r):
        """first sectors of rank 0's and the last rank's pieces vs the oracle
        (warmup round only, outside the timed region)"""
        torch.cuda.synchronize()
        n = min(4 * sector, chunk)
        ok = True
        send = pipe.send[r % len(pipe.send)]
        for g in (0, world - 1):
            a = g * piece_bytes
            src = send[a + H:a + H + n].cpu().numpy().tobytes()
            if decrypt:
                exp = cpu_ref.cbc(key, send[a:a + H].cpu().numpy().tobytes(), src, decrypt=True)
            else:
                exp = cpu_ref.cbc_segments(key, sh.ctr_add(iv0, (r * world + g) * chunk // sector), src, sector)
            ok = ok and gathered[a + H:a + H + n].cpu().numpy().tobytes() == exp
        if decrypt and world > 1:  # halo of rank 1 = last ciphertext block of rank 0
            ok = ok and torch.equal(send[piece_bytes:piece_bytes + H], send[piece_bytes - H:piece_bytes])
        verdict["ok"] = ok

    pipe.run(1, produce, work, verify)  # warmup + verification
    torch.cuda.synchronize()
    if pdist._pg_on():
        dist.barrier()
    t0 = time.perf_counter()
    pipe.run(rounds, produce, work)
    torch.cuda.synchronize()
    if pdist._pg_on():
        dist.barrier()
    el = pdist.allreduce_max(time.perf_counter() - t0)
    ok = pdist.allreduce_max(0.0 if verdict.get("ok", rank != 0) else 1.0) == 0.0
    total = rounds * chunk * world
    return {
        "seconds": el,
        "total_bytes": total,
        "gbps": total / el / 1e9 if el > 0 else 0.0,
        "verified": ok,
        "ranks": world,
        "backend": dist.get_backend() if pdist._pg_on() else "none",
        "collectives": bool(pipe.comm),
        "overlap": pipe.overlap,
        # bytes that cross xGMI: every non-root piece out (scatter) and back (gather)
        "xgmi_bytes": 2 * rounds * (world - 1) * piece_bytes,
    }
