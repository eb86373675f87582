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
from datetime import timedelta

import torch
import torch.distributed as dist

from ..models import cpu_ref
from . import shard as sh


def local_gpu() -> int:
    """The GPU this rank drives: LOCAL_RANK, or LOCAL_RANK mod the visible
    device count under OTC_SHARE_GPUS=1 (rehearsals with more ranks than
    GPUs).  Needs no process group, so callers can bind the device and create
    streams before RCCL creates its own."""
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        return local
    n = torch.cuda.device_count()
    if local >= n:
        if os.environ.get("OTC_SHARE_GPUS") != "1":
            raise RuntimeError(f"LOCAL_RANK {local} but only {n} GPU(s) visible (OTC_SHARE_GPUS=1 to share)")
        return local % n
    return local


def collective_timeout() -> timedelta:
    """Bound on any one collective of the default and duplex groups
    (OTC_COLLECTIVE_TIMEOUT_S, default 300 s; torch's default is 30 min).
    With TORCH_NCCL_ASYNC_ERROR_HANDLING=1 (set here unless the caller chose)
    torch's RCCL watchdog tears the rank down when one stalls past it, so a
    dead peer ends the job instead of hanging it -- the Python-side
    counterpart of the C job's ncclCommGetAsyncError poll
    (csrc/hip/pipeline.cpp).  The bench's collectives move <= 2 GiB per rank
    over xGMI (seconds at worst), so 300 s only trips on a real stall."""
    return timedelta(seconds=float(os.environ.get("OTC_COLLECTIVE_TIMEOUT_S", "300")))


def init_from_env(backend: str | None = None, force: bool = False):
    """Initialise the default process group from torchrun's env and bind the
    rank to its GPU.  Returns (rank, world, gpu): gpu = LOCAL_RANK (one
    process per GPU).

    Rehearsal knobs (multi-rank code paths on a box with fewer GPUs than
    ranks, e.g. 2 ranks on one MI355X): OTC_DIST_BACKEND=gloo picks the
    backend (RCCL refuses two ranks on one device) and OTC_SHARE_GPUS=1 maps
    rank r to GPU r mod device_count instead of failing; OTC_DIST_FORCE=1
    creates the process group even at world size 1 (so does ``force``; a
    missing MASTER_ADDR/MASTER_PORT then defaults to 127.0.0.1 and a free
    port)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    backend = backend or os.environ.get("OTC_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    gpu = local_gpu()
    if torch.cuda.is_available():
        torch.cuda.set_device(gpu)
    force = force or os.environ.get("OTC_DIST_FORCE") == "1"  # a 1-rank group too (exercises the RCCL path)
    if (world > 1 or force) and not dist.is_initialized():
        if world == 1:
            from .launch import free_port

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if backend == "nccl":
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
            dist.init_process_group(backend, device_id=torch.device("cuda", gpu), timeout=collective_timeout())
        else:
            dist.init_process_group(backend, timeout=collective_timeout())
    return rank, world, gpu


def _pg_on() -> bool:
    return dist.is_available() and dist.is_initialized()


def _world():
    if _pg_on():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def reset_groups():
    """Forget the cached duplex communicators (call after
    destroy_process_group, before initialising a new default group)."""
    _DUPLEX_GROUPS.clear()


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
    (shards in rank order, any sizes; all but the last a multiple of 16 bytes).

    The counter offset is this shard's byte offset / 16.  With
    ``global_nbytes`` the layout is taken to be ``shard.plan(global_nbytes,
    world)`` (checked against the local size) and no communication happens;
    otherwise the offset is the exclusive prefix sum of the local sizes (one
    small all_gather)."""
    rank, world = _world()
    n = local.numel() * local.element_size()
    if n % sh.BLOCK and rank != world - 1:
        raise ValueError("all shards but the last must be a multiple of 16 bytes")
    if global_nbytes is not None:
        s = sh.plan(global_nbytes, world)[rank]
        if s.nbytes != n:
            raise ValueError(f"rank {rank}: local shard has {n} bytes but plan({global_nbytes}, {world}) "
                             f"gives it {s.nbytes}")
        offset = s.offset
    elif world > 1:
        sizes = _all_gather_int(n)
        offset = sum(sizes[:rank])
        if any(v % sh.BLOCK for v in sizes[:-1]):
            raise ValueError("all shards but the last must be a multiple of 16 bytes")
    else:
        offset = 0
    return _ctr_local(local, key, counter, offset // sh.BLOCK, impl)


def _all_gather_int(v: int) -> list[int]:
    on_gpu = torch.cuda.is_available() and dist.get_backend() == "nccl"
    device = torch.device("cuda", torch.cuda.current_device()) if on_gpu else "cpu"
    t = torch.tensor([v], dtype=torch.int64, device=device)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [int(x.item()) for x in out]


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


_DUPLEX_GROUPS: dict = {}


def duplex_groups():
    """Two extra communicators over all ranks -- one carries scatters, the
    other gathers.  Each communicator has its own RCCL stream, so a gather
    (root ingress) and the next round's scatter (root egress) run at the same
    time: xGMI links are full duplex, and one communicator would serialise the
    two directions.  Collective on first use (every rank calls it in the same
    order); cached afterwards."""
    if not _pg_on():
        return None, None
    key = (dist.get_backend(), dist.get_world_size())
    if key not in _DUPLEX_GROUPS:
        _DUPLEX_GROUPS[key] = (dist.new_group(timeout=collective_timeout()), dist.new_group(timeout=collective_timeout()))
    return _DUPLEX_GROUPS[key]


class ScatterGatherPipeline:
    """Double-buffered root scatter -> per-rank work -> root gather.

    Round r: the root fills a ``world x chunk`` staging buffer (``produce``),
    scatters it (one ``chunk`` per rank), every rank runs ``fn(piece, out, r)``
    writing ``out``, and ``out`` is gathered back to the root, which hands it to
    ``consume``.  With ``overlap`` the gather of round r is asynchronous on its
    own communicator and overlaps the scatter + work of round r+1 (two buffer
    slots; a slot is reused only after the gather that read it has finished).

    Memory: 4 x chunk per rank, plus 4 x world x chunk on the root -- chunked
    rounds, so a stream larger than one GPU's 288 GB streams through the root.

    ``OTC_DUPLEX=0`` in the environment turns the overlap off for every
    pipeline of the process: scatter and gather then share the default
    group's one communicator, one after the other -- the fallback if two
    concurrent RCCL communicators per GPU ever misbehave on a node (RCCL
    allows it; each communicator's collectives are issued in the same order
    on every rank, so they cannot cross-wait).
    """

    def __init__(self, chunk_per_rank: int, root: int = 0, device=None, overlap: bool = True):
        self.rank, self.world = _world()
        self.root = root
        if device is None:
            device = (torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
                      else torch.device("cpu"))
        self.device = torch.device(device)
        self.chunk = max(sh.BLOCK, chunk_per_rank - chunk_per_rank % sh.BLOCK)
        # collectives whenever a process group exists, even at world size 1
        # (a 1-rank RCCL group runs the same scatter/gather code path)
        self.comm = _pg_on()
        self.overlap = overlap and self.comm and os.environ.get("OTC_DUPLEX", "1") != "0"
        self.g_sc, self.g_ga = duplex_groups() if self.overlap else (None, None)
        nslot = 2 if self.overlap else 1

        def mk(n):
            return torch.empty(n, dtype=torch.uint8, device=self.device)

        self.recv = [mk(self.chunk) for _ in range(nslot)]
        self.out = [mk(self.chunk) for _ in range(nslot)]
        is_root = self.rank == root
        self.send = [mk(self.chunk * self.world) for _ in range(nslot)] if is_root else None
        self.gath = [mk(self.chunk * self.world) for _ in range(nslot)] if is_root else None

    def _drain(self, pend, consume):
        work, slot, r = pend
        if work is not None:
            work.wait()
        if self.rank == self.root and consume is not None:
            consume(self.gath[slot], r)

    def run(self, nrounds: int, produce, fn, consume=None):
        """produce(send, r): root fills round r's staging buffer;
        fn(piece, out, r): every rank writes its result for round r to out;
        consume(gathered, r): root receives round r's gathered results."""
        is_root = self.rank == self.root
        nslot = len(self.recv)
        pending = [None] * nslot
        for r in range(nrounds):
            s = r % nslot
            if pending[s] is not None:  # the gather of round r - nslot still reads out[s]
                self._drain(pending[s], consume)
                pending[s] = None
            if is_root:
                produce(self.send[s], r)
            if self.comm:
                dist.scatter(self.recv[s], list(self.send[s].chunk(self.world)) if is_root else None,
                             src=self.root, group=self.g_sc)
            else:
                self.recv[s].copy_(self.send[s])
            fn(self.recv[s], self.out[s], r)
            if self.comm:
                work = dist.gather(self.out[s], list(self.gath[s].chunk(self.world)) if is_root else None,
                                   dst=self.root, group=self.g_ga, async_op=self.overlap)
            else:
                self.gath[s].copy_(self.out[s])
                work = None
            pending[s] = (work if self.overlap else None, s, r)
            if not self.overlap:
                self._drain(pending[s], consume)
                pending[s] = None
        for k in range(nrounds, nrounds + nslot):  # drain in round order
            s = k % nslot
            if pending[s] is not None:
                self._drain(pending[s], consume)
                pending[s] = None


def scatter_apply_gather(full: torch.Tensor | None, nbytes: int, fn, root: int = 0,
                         chunk_per_rank: int = 256 << 20, device=None, overlap: bool = True) -> torch.Tensor | None:
    """Root-resident stream -> equal-count chunked scatter -> ``fn(piece,
    global_byte_offset)`` on every rank -> gather back to the root, through
    ``ScatterGatherPipeline`` (the gather of round r overlaps the scatter of
    round r+1).  Streams larger than one GPU's HBM are processed in rounds.
    Returns the processed stream on the root (None elsewhere)."""
    rank, world = _world()
    if device is None and full is not None:
        device = full.device
    pipe = ScatterGatherPipeline(chunk_per_rank, root=root, device=device, overlap=overlap)
    chunk = pipe.chunk
    round_bytes = chunk * world
    nrounds = -(-nbytes // round_bytes)
    out = torch.empty(nbytes, dtype=torch.uint8, device=pipe.device) if rank == root else None
    flat = full.reshape(-1).view(torch.uint8) if full is not None else None

    def produce(send, r):
        off = r * round_bytes
        n = min(round_bytes, nbytes - off)
        send[:n].copy_(flat[off:off + n])
        if n < round_bytes:
            send[n:].zero_()

    def work(piece, dst, r):
        gofs = r * round_bytes + rank * chunk
        valid = max(0, min(chunk, nbytes - gofs))
        if valid:
            dst[:valid].copy_(fn(piece[:valid], gofs))

    def consume(gathered, r):
        off = r * round_bytes
        n = min(round_bytes, nbytes - off)
        out[off:off + n].copy_(gathered[:n])

    pipe.run(nrounds, produce, work, consume)
    return out


def scatter_ctr(full: torch.Tensor | None, nbytes: int, key: bytes, counter: bytes, root: int = 0,
                chunk_per_rank: int = 256 << 20, impl="auto", overlap: bool = True):
    """CTR over a root-resident stream via RCCL scatter/gather."""
    def fn(piece, gofs):
        return _ctr_local(piece, key, counter, gofs // sh.BLOCK, impl)

    return scatter_apply_gather(full, nbytes, fn, root=root, chunk_per_rank=chunk_per_rank, overlap=overlap)


def gather_floats(values: list[float]) -> list[list[float]]:
    """Every rank's short float list, on every rank (rank order); ``nan``
    stands for "not measured".  One all_gather of a float64 tensor."""
    if not _pg_on():
        return [list(map(float, values))]
    on_gpu = torch.cuda.is_available() and dist.get_backend() == "nccl"
    device = torch.device("cuda", torch.cuda.current_device()) if on_gpu else "cpu"
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    outs = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(outs, t)
    return [o.cpu().tolist() for o in outs]


def allreduce_max(value: float, device=None) -> float:
    if not _pg_on():
        return value
    if device is None:
        on_gpu = torch.cuda.is_available() and dist.get_backend() == "nccl"
        device = torch.device("cuda", torch.cuda.current_device()) if on_gpu else "cpu"
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
