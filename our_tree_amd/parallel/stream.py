"""Host-memory streaming through the native pinned pipeline (otc_engine_*:
H2D(k+1) | kernel(k) | D2H(k-1) on three HIP streams, csrc/hip/engine.cpp) and
the single-process multi-GPU planner (otc_multi_run: direct per-GPU ingest or
RCCL root scatter/gather over xGMI).

Replaces the reference's synchronous pageable cudaMemcpy around every launch
(/root/reference/aes-gpu/Source/AES.cu:230-282).
"""
from __future__ import annotations

import ctypes

import numpy as np

from .. import _native
from ..ops.aes_ops import _impl
from ..ops.keys import expand_key

MODES = {"ecb": 0, "ctr": 1, "cbc-dec": 2}
STRATEGIES = {"direct": 0, "rccl": 1}


def _ptr(a):
    if isinstance(a, np.ndarray):
        if not a.flags["C_CONTIGUOUS"]:
            raise ValueError("host buffers must be contiguous")
        return a.ctypes.data
    try:
        import torch

        if isinstance(a, torch.Tensor):
            if a.device.type != "cpu" or not a.is_contiguous():
                raise ValueError("host buffers must be contiguous CPU tensors")
            return a.data_ptr()
    except ImportError:
        pass
    raise TypeError("host buffer must be a numpy array or CPU tensor")


def _nb(a):
    return a.nbytes if isinstance(a, np.ndarray) else a.numel() * a.element_size()


class StreamEngine:
    """Pinned double/triple-buffered host<->GPU pipeline on one device."""

    def __init__(self, device: int = 0, chunk_bytes: int = 256 << 20, depth: int = 3, pooled_queues: bool = False):
        """``pooled_queues``: run the three streams on HIP's pooled hardware
        queues instead of queues of their own (otc_engine_create_ex; the A/B
        arm of docs/PERF.md "Round 6")."""
        self._lib = _native.require_gpu_lib()
        self._h = self._lib.otc_engine_create_ex(device, chunk_bytes, depth, 1 if pooled_queues else 0)
        if not self._h:
            _native.check(-5, "otc_engine_create")
        self.device = device

    def close(self):
        if self._h:
            self._lib.otc_engine_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def run(self, mode: str, host_in, host_out, key: bytes, iv_or_counter: bytes = bytes(16),
            block_offset: int = 0, impl: str = "auto") -> dict:
        n = _nb(host_in)
        if _nb(host_out) < n:
            raise ValueError("output buffer too small")
        k = expand_key(key, decrypt=(mode == "cbc-dec"))
        st = _native.StreamStats()
        ivb = (ctypes.c_uint8 * 16).from_buffer_copy(bytes(iv_or_counter))
        rc = self._lib.otc_engine_run(self._h, MODES[mode], _ptr(host_in), _ptr(host_out), n, ctypes.byref(k), ivb,
                                      block_offset, _impl(impl), ctypes.byref(st))
        _native.check(rc, "otc_engine_run")
        return {"total_ms": st.total_ms, "kernel_ms": st.kernel_ms, "h2d_ms": st.h2d_ms, "d2h_ms": st.d2h_ms,
                "host_stage_ms": st.host_stage_ms, "bytes": st.bytes, "chunks": st.chunks,
                "numa_node": st.numa_node, "gbps": st.bytes / (st.total_ms * 1e6) if st.total_ms else 0.0,
                # per-direction PCIe rates over the time the copies were in flight
                "h2d_gbps": st.bytes / (st.h2d_ms * 1e6) if st.h2d_ms else 0.0,
                "d2h_gbps": st.bytes / (st.d2h_ms * 1e6) if st.d2h_ms else 0.0}

    @property
    def numa_node(self) -> int:
        """NUMA node of this engine's pinned staging ring (-1: unknown)."""
        return self._lib.otc_engine_numa_node(self._h)

    def staging_ptr(self, slot: int = 0) -> int:
        """Address of staging slot ``slot`` (0 until a pageable run allocated it)."""
        return self._lib.otc_engine_staging(self._h, slot) or 0


PTR_HOST, PTR_PINNED, PTR_DEVICE = 0, 1, 2  # otc.h OTC_PTR_*


def pageable_buffers(*bufs) -> list[int]:
    """Indices of the host buffers in ``bufs`` that are NOT pinned (plain
    pageable memory: the runtime stages every async copy of them through a
    bounce buffer and the copy blocks the host thread)."""
    lib = _native.require_gpu_lib()
    return [i for i, b in enumerate(bufs) if lib.otc_ptr_kind(_ptr(b)) == PTR_HOST]


def multi_gpu_run(mode: str, host_in, host_out, key: bytes, iv_or_counter: bytes = bytes(16), ngpus: int = 1,
                  strategy: str = "direct", chunk_bytes: int = 256 << 20, impl: str = "auto") -> dict:
    """Single-process multi-GPU processing of one host-resident stream.

    strategy "rccl" funnels the whole stream through GPU 0's host link and
    enqueues every H2D / D2H from one thread: with pageable host buffers those
    copies block and the pipeline serialises, so a RuntimeWarning is raised
    (pin them: ``pinned_empty``).  "direct" stages pageable data through its
    own NUMA-placed pinned ring and needs no warning."""
    import warnings

    lib = _native.require_gpu_lib()
    if strategy == "rccl":
        bad = pageable_buffers(host_in, host_out)
        if bad:
            which = " and ".join(("host_in", "host_out")[i] for i in bad)
            verb = "are" if len(bad) > 1 else "is"
            warnings.warn(f"multi_gpu_run(strategy='rccl'): {which} {verb} pageable; the root's H2D/D2H copies "
                          "block and serialise the pipeline -- allocate with pinned_empty()", RuntimeWarning,
                          stacklevel=2)
    k = expand_key(key, decrypt=(mode == "cbc-dec"))
    st = _native.MultiStats()
    ivb = (ctypes.c_uint8 * 16).from_buffer_copy(bytes(iv_or_counter))
    rc = lib.otc_multi_run(ngpus, STRATEGIES[strategy], MODES[mode], _ptr(host_in), _ptr(host_out), _nb(host_in),
                           ctypes.byref(k), ivb, _impl(impl), chunk_bytes,
                           ctypes.byref(st))
    _native.check(rc, "otc_multi_run")
    return {"total_ms": st.total_ms, "gbps": st.gbps, "ngpus": st.ngpus, "strategy": strategy,
            "numa_nodes_used": st.numa_nodes_used}


def multi_ctr_resident(bufs, key: bytes, counter: bytes, impl: str = "auto") -> float:
    """In-place CTR over device-resident shards ``bufs[g]`` (on GPU g, equal
    sizes, shard g at counter offset g * shard_blocks), all GPUs concurrently
    from one host thread (otc_multi_ctr_resident).  Returns elapsed ms."""
    lib = _native.require_gpu_lib()
    if not bufs:
        raise ValueError("bufs must hold one tensor per GPU")
    # shard size in BYTES (any dtype): the native call and the per-shard
    # counter offset g * n / 16 both count bytes
    n = bufs[0].numel() * bufs[0].element_size()
    for g, b in enumerate(bufs):
        if not b.is_cuda or b.device.index != g or not b.is_contiguous():
            raise ValueError("bufs[g] must be a contiguous tensor on cuda:g")
        if b.numel() * b.element_size() != n:
            raise ValueError("every shard must have the same byte size")
    if n % 16:
        raise ValueError(f"shard byte size must be a multiple of 16 (got {n})")
    ptrs = (ctypes.c_void_p * len(bufs))(*[b.data_ptr() for b in bufs])
    k = expand_key(key)
    ms = ctypes.c_double()
    ivb = (ctypes.c_uint8 * 16).from_buffer_copy(bytes(counter))
    rc = lib.otc_multi_ctr_resident(len(bufs), ptrs, n, ctypes.byref(k), ivb, _impl(impl), ctypes.byref(ms))
    _native.check(rc, "otc_multi_ctr_resident")
    return ms.value


class _PinnedOwner:
    """Frees a hipHostMalloc allocation when the last numpy view dies."""

    def __init__(self, lib, ptr):
        self._lib, self.ptr = lib, ptr

    def __del__(self):
        try:
            self._lib.otc_host_free_pinned(self.ptr)
        except Exception:
            pass


def pinned_empty(nbytes: int) -> np.ndarray:
    """A uint8 numpy array over pinned (hipHostMalloc) host memory, so the
    engine copies it with DMA directly (no staging)."""
    lib = _native.require_gpu_lib()
    p = lib.otc_host_alloc_pinned(nbytes)
    if not p:
        raise MemoryError("hipHostMalloc failed")
    buf = (ctypes.c_uint8 * nbytes).from_address(p)
    buf._owner = _PinnedOwner(lib, p)  # lifetime: numpy view -> ctypes buffer -> owner
    return np.frombuffer(buf, dtype=np.uint8)
