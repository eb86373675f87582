"""One-process-per-GPU data parallelism over torch.distributed.

On MI355X the ``nccl`` backend IS RCCL; collectives run over xGMI.  The cipher
workloads map onto three communication patterns:

* **Resident DP (CTR/ECB)**: every rank owns a contiguous shard and encrypts it
  with its own counter offset -- zero communication in steady state.
* **Root scatter / gather** (``scatter_apply_gather``): plaintext resident on
  one GPU is scattered in equal-count, chunk-pipelined pieces (RCCL scatter is a
  one-hop fan-out from the root over its 7 xGMI links), processed, gathered.
* **CBC-decrypt halo exchange** (``cbc_decrypt_sharded``): each rank needs the
  last ciphertext block of its left neighbour -- a 16-byte send/recv ring step,
  the cipher analog of ring-attention's neighbour exchange.

CPU tensors (gloo backend) are processed with the C oracle, so the whole
distribution logic is testable without a GPU.  The reference had no multi-device
code at all.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from ..models import cpu_ref
from . import shard as sh


def init_from_env(backend: str | None = None):
    """Initialise the default process group from torchrun's env; binds the
    rank to LOCAL_RANK's GPU.  Returns (rank, world, local_rank)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    elif torch.cuda.is_available():
        torch.cuda.set_device(local)
    return rank, world, local


def _world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _ctr_local(x: torch.Tensor, key: bytes, counter: bytes, block_offset: int, impl="auto") -> torch.Tensor:
    if x.device.type == "cuda":
        from .. import ops

        return ops.ctr(x, key, counter, out=x, block_offset=block_offset, impl=impl)
    data = x.numpy().tobytes()
    res = cpu_ref.ctr(key, counter, data, block_offset)
    x.copy_(torch.frombuffer(bytearray(res), dtype=torch.uint8).view_as(x))
    return x


def sharded_ctr_(local: torch.Tensor, key: bytes, counter: bytes, global_nbytes: int | None = None,
                 impl="auto") -> torch.Tensor:
    """In-place CTR on this rank's shard of a globally contiguous stream
    (equal-size shards in rank order; the counter offset is derived from the
    rank).  No communication."""
    rank, world = _world()
    n = local.numel() * local.element_size()
    if n % sh.BLOCK and rank != world - 1:
        raise ValueError("all shards but the last must be a multiple of 16 bytes")
    return _ctr_local(local, key, counter, rank * (n // sh.BLOCK), impl)


def cbc_decrypt_sharded(local_ct: torch.Tensor, key: bytes, iv: bytes) -> torch.Tensor:
    """CBC decryption of this rank's contiguous ciphertext shard.  The halo
    (left neighbour's last ciphertext block) arrives by a ring send/recv."""
    rank, world = _world()
    flat = local_ct.reshape(-1).view(torch.uint8)
    if flat.numel() % sh.BLOCK:
        raise ValueError("CBC shards must be a multiple of 16 bytes")
    halo = torch.empty(sh.BLOCK, dtype=torch.uint8, device=flat.device)
    if world > 1:
        ops_ = []
        if rank + 1 < world:
            ops_.append(dist.P2POp(dist.isend, flat[-sh.BLOCK:].contiguous(), rank + 1))
        if rank > 0:
            ops_.append(dist.P2POp(dist.irecv, halo, rank - 1))
        if ops_:
            for req in dist.batch_isend_irecv(ops_):
                req.wait()
    my_iv = bytes(iv) if rank == 0 else bytes(halo.cpu().numpy().tobytes())
    if flat.device.type == "cuda":
        from .. import ops

        return ops.cbc_decrypt(flat, key, my_iv).view_as(local_ct)
    res = cpu_ref.cbc(key, my_iv, flat.numpy().tobytes(), decrypt=True)
    return torch.frombuffer(bytearray(res), dtype=torch.uint8).view_as(local_ct)


def scatter_apply_gather(full: torch.Tensor | None, nbytes: int, fn, root: int = 0,
                         chunk_per_rank: int = 256 << 20, device=None) -> torch.Tensor | None:
    """Root-resident stream -> equal-count chunked scatter -> ``fn(piece,
    global_byte_offset)`` on every rank -> gather back to the root.

    Only 2 x chunk_per_rank of scratch is needed per rank and
    world x chunk_per_rank on the root, so streams larger than one GPU's
    HBM can be processed in rounds.  Returns the processed stream on the root
    (None elsewhere)."""
    rank, world = _world()
    if device is None:
        device = full.device if full is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
    chunk_per_rank = max(sh.BLOCK, chunk_per_rank - chunk_per_rank % sh.BLOCK)
    round_bytes = chunk_per_rank * world
    out = torch.empty(nbytes, dtype=torch.uint8, device=device) if rank == root else None
    recv = torch.empty(chunk_per_rank, dtype=torch.uint8, device=device)
    flat = full.reshape(-1).view(torch.uint8) if full is not None else None
    for off in range(0, nbytes, round_bytes):
        n = min(round_bytes, nbytes - off)
        if rank == root:
            pieces = []
            for r in range(world):
                p = torch.zeros(chunk_per_rank, dtype=torch.uint8, device=device)
                a, b = off + r * chunk_per_rank, min(off + (r + 1) * chunk_per_rank, off + n)
                if b > a:
                    p[: b - a].copy_(flat[a:b])
                pieces.append(p)
        else:
            pieces = None
        if world > 1:
            dist.scatter(recv, pieces if rank == root else None, src=root)
        else:
            recv.copy_(pieces[0])
        gofs = off + rank * chunk_per_rank
        valid = max(0, min(chunk_per_rank, nbytes - gofs))
        if valid:
            recv[:valid] = fn(recv[:valid].contiguous(), gofs)
        gathered = [torch.empty_like(recv) for _ in range(world)] if rank == root else None
        if world > 1:
            dist.gather(recv, gathered, dst=root)
        else:
            gathered = [recv.clone()]
        if rank == root:
            for r in range(world):
                a, b = off + r * chunk_per_rank, min(off + (r + 1) * chunk_per_rank, off + n)
                if b > a:
                    out[a:b].copy_(gathered[r][: b - a])
    return out


def scatter_ctr(full: torch.Tensor | None, nbytes: int, key: bytes, counter: bytes, root: int = 0,
                chunk_per_rank: int = 256 << 20, impl="auto"):
    """CTR over a root-resident stream via RCCL scatter/gather."""
    def fn(piece, gofs):
        return _ctr_local(piece, key, counter, gofs // sh.BLOCK, impl)

    return scatter_apply_gather(full, nbytes, fn, root=root, chunk_per_rank=chunk_per_rank)


def allreduce_max(value: float, device=None) -> float:
    rank, world = _world()
    if world == 1:
        return value
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
