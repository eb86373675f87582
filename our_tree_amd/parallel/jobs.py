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

Verification is per rank and observed, not assumed (``check_round``): after
the warmup round and after the last timed round, every rank checksums the
piece it RECEIVED and the piece it PRODUCED and checks a sample of its own
output against the C oracle; the root compares those checksums with the
slices it sent and the slices it gathered.  A rank counts as verified only if
all three agree in both rounds, and the bytes reported as moved over xGMI are
the bytes of those verified non-root pieces.  The reference had no
multi-device code to compare against; its worker sweep is
/root/reference/test.c:135-153.

The job runs on CUDA tensors (RCCL) or CPU tensors (gloo + the C oracle), so
the whole protocol, fault injection included, is tested without a GPU
(tests/test_jobs_cpu.py).
"""
from __future__ import annotations

import time

import numpy as np
import torch
import torch.distributed as dist

from ..models import cpu_ref
from . import dist as pdist
from . import shard as sh

_CSUM_MUL = 0x9E3779B97F4A7C15 | 1


def checksum(t: torch.Tensor) -> int:
    """Position-dependent 64-bit XOR fold of a byte buffer (size % 8 == 0):
    XOR over words i of (w_i * 0x9E3779B97F4A7C15 + 2i) mod 2^64.  The device
    kernel (``ops.checksum``, csrc/hip/stream_ops.hip k_checksum_kernel) and
    this host version compute the same value."""
    if t.device.type == "cuda":
        from .. import ops

        return ops.checksum(t)
    b = t.contiguous().view(torch.uint8).numpy()
    if b.size % 8:
        raise ValueError("checksum needs a multiple of 8 bytes")
    w = b.view("<u8")
    i = np.arange(w.size, dtype=np.uint64)
    return int(np.bitwise_xor.reduce(w * np.uint64(_CSUM_MUL) + (i << np.uint64(1)), initial=np.uint64(0)))


def _fill(t: torch.Tensor, seed: int):
    if t.device.type == "cuda":
        from .. import ops

        ops.fill_random_(t, seed=seed)
    else:
        g = torch.Generator().manual_seed(seed)
        t.copy_(torch.randint(0, 256, t.shape, dtype=torch.uint8, generator=g))


def _put(dst: torch.Tensor, data: bytes):
    dst.copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))


def _cbc_segments(x, key, iv, sector, out):
    if x.device.type == "cuda":
        from .. import ops

        ops.cbc_encrypt_segments(x, key, iv, sector, out=out)
    else:
        _put(out, cpu_ref.cbc_segments(key, iv, x.numpy().tobytes(), sector))


def _cbc_decrypt(x, key, iv, out):
    if x.device.type == "cuda":
        from .. import ops

        ops.cbc_decrypt(x, key, iv, out=out)
    else:
        _put(out, cpu_ref.cbc(key, iv, x.numpy().tobytes(), decrypt=True))


def _gather_i64(vals: list[int], device) -> list[list[int]]:
    """All-gather a short list of 64-bit values from every rank."""
    rank, world = pdist._world()
    t = torch.tensor([v - (1 << 64) if v >= (1 << 63) else v for v in vals], dtype=torch.int64, device=device)
    if not pdist._pg_on():
        outs = [t]
    else:
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t)
    return [[int(x) & (2**64 - 1) for x in o.cpu().tolist()] for o in outs]


def _comm_device():
    """where small verdict tensors live: the GPU under RCCL, else the host"""
    if pdist._pg_on() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def check_round(pipe, slot: int, r: int, work_ok) -> list[bool]:
    """Collective: per-rank verdict of the round whose buffers sit in ``slot``.
    Every rank checksums its received and produced piece and runs
    ``work_ok(recv, out, r)`` (its own oracle sample); the root compares the
    checksums with the slices it sent and gathered.  Returns, on every rank,
    ``ok[g]`` for every rank g."""
    rank, world = pdist._world()
    recv, out = pipe.recv[slot], pipe.out[slot]
    if recv.device.type == "cuda":
        torch.cuda.synchronize(recv.device)
    mine = [checksum(recv), checksum(out), 1 if work_ok(recv, out, r) else 0]
    dev = _comm_device()
    allv = _gather_i64(mine, dev)
    flags = torch.zeros(world, dtype=torch.int64, device=dev)
    if rank == pipe.root:
        sent = [checksum(c) for c in pipe.send[slot].chunk(world)]
        got = [checksum(c) for c in pipe.gath[slot].chunk(world)]
        for g in range(world):
            s_ok, w_ok, g_ok = allv[g][0] == sent[g], allv[g][2] == 1, allv[g][1] == got[g]
            flags[g] = 1 if (s_ok and w_ok and g_ok) else 0
    if pdist._pg_on():
        dist.broadcast(flags, src=pipe.root)
    return [bool(v) for v in flags.cpu().tolist()]


def cbc_scatter_job(rounds: int, chunk: int, key: bytes, iv0: bytes, sector: int = 4096, decrypt: bool = False,
                    overlap: bool = True, device=None, fault: tuple | None = None) -> dict:
    """Run 1 verified warmup round + ``rounds`` timed rounds (the last one
    verified after the clock stops); every rank gets ``chunk`` bytes per
    round.  Returns (on every rank) a dict with the timing, the per-rank
    verdicts and the bytes observed to cross between GPUs.

    ``fault`` = (rank, "recv" | "out"): testing hook that flips one byte of
    that rank's received piece (a transport fault) or of its output (a
    compute fault, inside the oracle-checked sample) in the warmup round."""
    rank, world = pdist._world()
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
    device = torch.device(device)
    H = 16 if decrypt else 0
    piece_bytes = chunk + H
    pipe = pdist.ScatterGatherPipeline(piece_bytes, root=0, device=device, overlap=overlap)
    if pipe.chunk != piece_bytes:
        raise ValueError(f"chunk must be a positive multiple of 16 bytes (got {chunk})")
    carry = torch.tensor(list(iv0), dtype=torch.uint8, device=device)

    def produce(send, r):
        if not decrypt:
            _fill(send, r)
            return
        v = send.view(world, piece_bytes)
        for g in range(world):  # synthetic ciphertext, piece by piece (rows are strided)
            _fill(v[g, H:], r * world + g)
        v[0, :H].copy_(carry)
        v[1:, :H].copy_(v[:-1, -H:])
        carry.copy_(v[-1, -H:])

    def work(piece, out, r):
        if fault is not None and r == 0 and fault[0] == rank and fault[1] == "recv":
            piece[H + 7].bitwise_xor_(torch.tensor(0x5A, dtype=torch.uint8, device=piece.device))
        if not decrypt:
            gofs = (r * world + rank) * chunk
            _cbc_segments(piece, key, sh.ctr_add(iv0, gofs // sector), sector, out)
        else:
            # IV 0, then XOR the halo into the first block: no host round trip
            _cbc_decrypt(piece[H:], key, bytes(16), out[H:])
            out[H:2 * H].bitwise_xor_(piece[:H])
            out[:H].copy_(piece[:H])
        if fault is not None and r == 0 and fault[0] == rank and fault[1] == "out":
            out[H + 9].bitwise_xor_(torch.tensor(0xA5, dtype=torch.uint8, device=out.device))

    n_sample = min(4 * sector, chunk)

    def work_ok(recv, out, r):
        """this rank's output sample vs the C oracle run on what it received"""
        src = recv[H:H + n_sample].cpu().numpy().tobytes()
        if decrypt:
            exp = cpu_ref.cbc(key, recv[:H].cpu().numpy().tobytes(), src, decrypt=True)
        else:
            exp = cpu_ref.cbc_segments(key, sh.ctr_add(iv0, (r * world + rank) * chunk // sector), src, sector)
        return out[H:H + n_sample].cpu().numpy().tobytes() == exp

    halo_ok = [True]

    def consume_first(gathered, r):
        # exact-decrypt halo of rank 1 = last ciphertext block of rank 0's piece
        if decrypt and world > 1:
            send = pipe.send[0]
            halo_ok[0] = torch.equal(send[piece_bytes:piece_bytes + H], send[piece_bytes - H:piece_bytes])

    pipe.run(1, produce, work, consume_first)  # warmup round, slot 0
    ok_warm = check_round(pipe, 0, 0, work_ok)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    if pdist._pg_on():
        dist.barrier()
    t0 = time.perf_counter()
    pipe.run(rounds, produce, work)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    if pdist._pg_on():
        dist.barrier()
    el = pdist.allreduce_max(time.perf_counter() - t0)
    ok_last = check_round(pipe, (rounds - 1) % len(pipe.recv), rounds - 1, work_ok) if rounds > 0 else ok_warm
    per_rank = [a and b for a, b in zip(ok_warm, ok_last)]
    halo = pdist.allreduce_max(0.0 if halo_ok[0] else 1.0) == 0.0
    nver = sum(per_rank)
    total = rounds * chunk * world
    # bytes that demonstrably crossed between GPUs: every verified non-root
    # piece out (scatter) and back (gather), in the two checked rounds
    peer_verified = sum(2 * piece_bytes * (2 if rounds > 0 else 1)
                        for g, ok in enumerate(per_rank) if ok and g != pipe.root) if pipe.comm else 0
    # what the timed collectives were asked to move between ranks (their last
    # round is among the verified ones above)
    peer_timed = 2 * rounds * (world - 1) * piece_bytes if pipe.comm else 0
    backend = dist.get_backend() if pdist._pg_on() else "none"
    # only RCCL ("nccl") moves GPU-to-GPU bytes over xGMI; gloo (the CPU
    # rehearsals) moves them through host memory / TCP
    xgmi = backend == "nccl"
    return {
        "seconds": el,
        "total_bytes": total,
        "gbps": total / el / 1e9 if el > 0 else 0.0,
        "verified": nver == world and halo,
        "ranks": world,
        "ranks_verified": nver,
        "per_rank_ok": per_rank,
        "backend": backend,
        "collectives": bool(pipe.comm),
        "overlap": pipe.overlap,
        # a 1-rank group moves nothing between GPUs: its "scatter" is a local copy
        "transport": ("local" if world == 1 else "xgmi" if xgmi else "host") if pipe.comm else "none",
        "peer_bytes_verified": peer_verified,
        "peer_bytes_timed": peer_timed,
        "xgmi_bytes_verified": peer_verified if xgmi else 0,
        "xgmi_bytes_timed": peer_timed if xgmi else 0,
        "host_bytes_verified": 0 if xgmi else peer_verified,
        "host_bytes_timed": 0 if xgmi else peer_timed,
    }
