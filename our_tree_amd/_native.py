"""ctypes bindings to the in-tree native libraries.

* ``lib/libotc.so``      -- gfx950 HIP kernels + C++ runtime + CPU oracle
                            (built by ``make`` / ``__graft_entry__.build()``)
* ``lib/libotc_cpu.so``  -- CPU oracle only (no ROCm dependency)

The GPU library is loaded AFTER ``torch`` so that it binds to the HIP runtime
torch already mapped (both carry SONAME ``libamdhip64.so.7``) and streams are
shared.  Loading fails loudly: there is no silent Python fallback for device
ops (see ``require_gpu_lib``).

C API: ``csrc/include/otc.h`` (device ops, engine, multi-GPU) and the
reference-compatible ``aes.h`` / ``arc4.h`` / ``rc4.h`` / ``aesni.h``
(parity with /root/reference/aes-modes/aes.h:62-161, /root/reference/arc4.h:54-77).
"""
from __future__ import annotations

import atexit
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")
# OTC_LIB selects a variant build of the same library for A/B measurements
# (``make variant NAME=x VFLAGS=-D...`` -> variants/x/libotc.so); default: the in-tree build
GPU_LIB_PATH = os.environ.get("OTC_LIB") or os.path.join(LIB_DIR, "libotc.so")
CPU_LIB_PATH = os.path.join(LIB_DIR, "libotc_cpu.so")

_lock = threading.Lock()
_gpu_lib = None
_cpu_lib = None

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_vp = ctypes.c_void_p
c_sz = ctypes.c_size_t
c_u64 = ctypes.c_uint64
c_int = ctypes.c_int


class OtcAesKey(ctypes.Structure):
    """Mirror of ``otc_aes_key`` (otc.h): expanded key passed by value to kernels."""

    _fields_ = [
        ("rk", ctypes.c_uint32 * 60),
        ("nr", ctypes.c_int32),
        ("dir", ctypes.c_int32),
        ("bits", ctypes.c_int32),
        ("pad", ctypes.c_int32),
    ]


class AesContext(ctypes.Structure):
    """Mirror of the reference-compatible ``aes_context`` {nr, rk, buf[68]}."""

    _fields_ = [
        ("nr", ctypes.c_int),
        ("rk", ctypes.POINTER(ctypes.c_ulong)),
        ("buf", ctypes.c_ulong * 68),
    ]


class Arc4Context(ctypes.Structure):
    """Mirror of ``arc4_context`` {x, y, m[256]} (reference arc4.h:35-41)."""

    _fields_ = [("x", ctypes.c_int), ("y", ctypes.c_int), ("m", ctypes.c_uint8 * 256)]


class Rc4State(ctypes.Structure):
    """Mirror of ``struct rc4_state`` (reference rc4.h:43-47)."""

    _fields_ = [("perm", ctypes.c_char * 256), ("index1", ctypes.c_int), ("index2", ctypes.c_int)]


class OtcCtrCtx(ctypes.Structure):
    """Mirror of ``otc_aes_ctr_ctx`` (PolarSSL CTR resume state,
    reference aes-modes/aes.c:869-900)."""

    _fields_ = [("nonce_counter", ctypes.c_uint8 * 16), ("stream_block", ctypes.c_uint8 * 16),
                ("nc_off", ctypes.c_size_t)]


class StreamStats(ctypes.Structure):
    _fields_ = [
        ("total_ms", ctypes.c_double),
        ("kernel_ms", ctypes.c_double),
        ("h2d_ms", ctypes.c_double),
        ("d2h_ms", ctypes.c_double),
        ("host_stage_ms", ctypes.c_double),
        ("bytes", ctypes.c_size_t),
        ("chunks", ctypes.c_int),
        ("numa_node", ctypes.c_int),
    ]


class RcclPiece(ctypes.Structure):
    """otc_rccl_piece (otc.h): one GPU's piece of one round of the RCCL job"""
    _fields_ = [
        ("round_off", ctypes.c_uint64),
        ("round_bytes", ctypes.c_uint64),
        ("pad_bytes", ctypes.c_uint64),
        ("off", ctypes.c_uint64),
        ("bytes", ctypes.c_uint64),
        ("blk0", ctypes.c_uint64),
        ("halo", ctypes.c_int64),
    ]


class MultiStats(ctypes.Structure):
    _fields_ = [
        ("total_ms", ctypes.c_double),
        ("gbps", ctypes.c_double),
        ("ngpus", ctypes.c_int),
        ("strategy", ctypes.c_int),
        ("numa_nodes_used", ctypes.c_int),
    ]


def _declare_cpu(lib):
    P = ctypes.POINTER
    sig = {
        "aes_setkey_enc": (c_int, [P(AesContext), c_u8p, ctypes.c_uint]),
        "aes_setkey_dec": (c_int, [P(AesContext), c_u8p, ctypes.c_uint]),
        "aes_crypt_ecb": (c_int, [P(AesContext), c_int, c_u8p, c_u8p]),
        "aes_crypt_cbc": (c_int, [P(AesContext), c_int, c_sz, c_u8p, c_u8p, c_u8p]),
        "aes_crypt_cfb128": (c_int, [P(AesContext), c_int, c_sz, P(c_int), c_u8p, c_u8p, c_u8p]),
        "aes_crypt_ctr": (c_int, [P(AesContext), c_int, P(c_int), c_u8p, c_u8p, c_u8p, c_u8p]),
        "aes_self_test": (c_int, [c_int]),
        "aes_export_rk32": (c_int, [P(AesContext), P(ctypes.c_uint32)]),
        "aes_ctr_bulk": (c_int, [P(AesContext), c_u8p, c_u8p, c_u8p, c_sz, c_int]),
        "aes_ecb_bulk": (c_int, [P(AesContext), c_int, c_u8p, c_u8p, c_sz, c_int]),
        "aes_ctr128_add": (None, [c_u8p, c_u64]),
        "arc4_setup": (None, [P(Arc4Context), c_u8p, ctypes.c_uint]),
        "arc4_prep": (c_int, [P(Arc4Context), c_sz, c_u8p]),
        "arc4_crypt": (c_int, [c_sz, c_u8p, c_u8p, c_u8p]),
        "arc4_crypt_mt": (c_int, [c_sz, c_u8p, c_u8p, c_u8p, c_int]),
        "arc4_self_test": (c_int, [c_int]),
        "rc4_init": (None, [P(Rc4State), ctypes.c_char_p, c_int]),
        "rc4_crypt": (None, [P(Rc4State), ctypes.c_char_p, ctypes.c_char_p, c_int]),
        "CheckAESSupport": (c_int, []),
        "AES_128_Key_Expansion": (None, [c_u8p, c_u8p]),
        "AES_192_Key_Expansion": (None, [c_u8p, c_u8p]),
        "AES_256_Key_Expansion": (None, [c_u8p, c_u8p]),
        "AES_Key_Expansion_Dec": (None, [c_u8p, c_u8p, c_int]),
        "AES_ECB_encrypt": (None, [c_u8p, c_u8p, ctypes.c_ulong, c_u8p, c_int]),
        "AES_ECB_decrypt": (None, [c_u8p, c_u8p, ctypes.c_ulong, c_u8p, c_int]),
        "AES_CTR_encrypt": (None, [c_u8p, c_u8p, c_u8p, c_u8p, ctypes.c_ulong, c_u8p, c_int]),
        "AES_CTR_encrypt_at": (None, [c_u8p, c_u8p, c_u8p, c_u8p, ctypes.c_ulong, c_u8p, c_int, ctypes.c_ulonglong]),
        "otc_bitslice_selftest": (c_int, [c_int]),
        "otc_rccl_nrounds": (c_u64, [c_u64, c_int, c_u64]),
        "otc_rccl_plan_piece": (c_int, [c_u64, c_int, c_u64, c_u64, c_int, P(RcclPiece)]),
        "otc_rccl_halo_start": (c_u64, [c_u64, c_u64, c_u64]),
        "AES_CBC_encrypt": (None, [c_u8p, c_u8p, c_u8p, ctypes.c_ulong, c_u8p, c_int]),
        "AES_CFB128_encrypt": (None, [c_u8p, c_u8p, c_u8p, ctypes.c_ulong, c_u8p, c_int]),
        "aes_monte_carlo": (c_int, [c_int, c_int, c_u8p]),
        "aes_monte_carlo_expected": (ctypes.c_char_p, [c_int, c_int]),
        "otc_parse_cpulist": (c_int, [ctypes.c_char_p, c_u8p, c_int]),
        "otc_numa_node_of_pci": (c_int, [ctypes.c_char_p, ctypes.c_char_p]),
        "otc_numa_node_cpus": (c_int, [ctypes.c_char_p, c_int, c_u8p, c_int]),
        "otc_numa_num_nodes": (c_int, [ctypes.c_char_p]),
        "otc_numa_bind_thread": (c_int, [c_int]),
        "otc_numa_alloc": (c_vp, [c_sz, c_int]),
        "otc_numa_free": (None, [c_vp, c_sz]),
        "otc_numa_node_of_addr": (c_int, [c_vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def _declare_gpu(lib):
    _declare_cpu(lib)
    P = ctypes.POINTER
    K = P(OtcAesKey)
    sig = {
        "otc_last_error": (ctypes.c_char_p, []),
        "otc_pick_impl": (c_int, [c_int, c_int, c_int, c_u64]),
        "otc_last_impl": (c_int, []),
        "otc_split_stats": (None, [c_int]),
        "otc_split_fallback_reason": (ctypes.c_char_p, []),
        "otc_split_last_units": (c_int, [ctypes.POINTER(c_u64), ctypes.POINTER(c_u64), ctypes.POINTER(c_u64)]),
        "otc_aes_key_init": (c_int, [K, c_u8p, c_int, c_int]),
        "otc_aes_ecb": (c_int, [c_vp, c_vp, c_sz, K, c_int, c_vp]),
        "otc_aes_ctr": (c_int, [c_vp, c_vp, c_sz, K, c_u8p, c_u64, c_int, c_vp]),
        "otc_aes_ctr_rfc3686": (c_int, [c_vp, c_vp, c_sz, K, c_u8p, c_u8p, c_u64, c_int, c_vp]),
        "otc_aes_ctr_ctx_init": (c_int, [P(OtcCtrCtx), c_u8p]),
        "otc_aes_ctr_stream": (c_int, [P(OtcCtrCtx), K, c_sz, c_vp, c_vp, c_int, c_vp]),
        "otc_aes_cbc_decrypt": (c_int, [c_vp, c_vp, c_sz, K, c_u8p, c_vp]),
        "otc_aes_cbc_decrypt_impl": (c_int, [c_vp, c_vp, c_sz, K, c_u8p, c_int, c_vp]),
        "otc_stream_create": (c_vp, []),
        "otc_dev_malloc": (c_vp, [c_sz]),
        "otc_dev_free": (None, [c_vp]),
        "otc_memcpy": (c_int, [c_vp, c_vp, c_sz, c_int]),
        "otc_stream_destroy": (None, [c_vp]),
        "otc_stream_join": (c_int, [c_vp, c_vp]),
        "otc_aes_cbc_encrypt_segments": (c_int, [c_vp, c_vp, c_sz, c_sz, K, c_u8p, c_vp]),
        "otc_aes_cbc_encrypt_segments_impl": (c_int, [c_vp, c_vp, c_sz, c_sz, K, c_u8p, c_int, c_vp]),
        "otc_aes_cfb128_encrypt_segments_impl": (c_int, [c_vp, c_vp, c_sz, c_sz, K, c_u8p, c_int, c_vp]),
        "otc_aes_cbc_decrypt_segments": (c_int, [c_vp, c_vp, c_sz, c_sz, K, c_u8p, c_vp]),
        "otc_aes_cfb128_decrypt": (c_int, [c_vp, c_vp, c_sz, K, c_u8p, c_vp]),
        "otc_aes_cfb128_decrypt_impl": (c_int, [c_vp, c_vp, c_sz, K, c_u8p, c_int, c_vp]),
        "otc_aes_cfb128_encrypt_segments": (c_int, [c_vp, c_vp, c_sz, c_sz, K, c_u8p, c_vp]),
        "otc_aes_cfb128_decrypt_segments": (c_int, [c_vp, c_vp, c_sz, c_sz, K, c_u8p, c_vp]),
        "otc_aes_cfb128_decrypt_segments_impl": (c_int, [c_vp, c_vp, c_sz, c_sz, K, c_u8p, c_int, c_vp]),
        "otc_aes_cbc_decrypt_segments_impl": (c_int, [c_vp, c_vp, c_sz, c_sz, K, c_u8p, c_int, c_vp]),
        "otc_aes_ctr_batch": (c_int, [c_vp, c_vp, c_vp, c_vp, c_u64, c_int, c_int, c_vp]),
        "otc_xor": (c_int, [c_vp, c_vp, c_vp, c_sz, c_vp]),
        "otc_rc4_multi": (c_int, [c_vp, c_int, c_sz, c_sz, c_sz, c_vp, c_vp, c_vp]),
        "otc_rc4_crypt_batch": (c_int, [c_vp, c_sz, c_sz, c_vp, c_vp, c_vp]),
        "otc_fill_random": (c_int, [c_vp, c_sz, c_u64, c_vp]),
        "otc_checksum": (c_int, [c_vp, c_sz, c_vp, c_vp]),
        "otc_clock_probe": (c_int, [c_vp, ctypes.c_double, ctypes.c_double, c_vp]),
        "otc_AES_ECB_encrypt": (c_int, [c_vp, c_vp, ctypes.c_ulong, c_u8p, c_int, c_vp]),
        "otc_AES_ECB_decrypt": (c_int, [c_vp, c_vp, ctypes.c_ulong, c_u8p, c_int, c_vp]),
        "otc_AES_CTR_encrypt": (c_int, [c_vp, c_vp, c_u8p, c_u8p, ctypes.c_ulong, c_u8p, c_int, c_vp]),
        "otc_multi_release": (None, []),
        "otc_release_resources": (None, []),
        "otc_fault_inject_alloc": (None, [ctypes.c_long]),
        "otc_device_numa_node": (c_int, [c_int]),
        "otc_engine_numa_node": (c_int, [c_vp]),
        "otc_engine_staging": (c_vp, [c_vp, c_int]),
        "otc_device_count": (c_int, []),
        "otc_device_cus": (c_int, [c_int]),
        "otc_device_clock_khz": (c_int, [c_int]),
        "otc_set_device": (c_int, [c_int]),
        "otc_device_sync": (c_int, []),
        "otc_host_register": (c_int, [c_vp, c_sz]),
        "otc_host_unregister": (c_int, [c_vp]),
        "otc_host_alloc_pinned": (c_vp, [c_sz]),
        "otc_ptr_kind": (c_int, [c_vp]),
        "otc_host_free_pinned": (None, [c_vp]),
        "otc_engine_create": (c_vp, [c_int, c_sz, c_int]),
        "otc_engine_create_ex": (c_vp, [c_int, c_sz, c_int, c_int]),
        "otc_engine_destroy": (None, [c_vp]),
        "otc_engine_run": (c_int, [c_vp, c_int, c_vp, c_vp, c_sz, K, c_u8p, c_u64, c_int, P(StreamStats)]),
        "otc_multi_run": (c_int, [c_int, c_int, c_int, c_vp, c_vp, c_sz, K, c_u8p, c_int, c_sz, P(MultiStats)]),
        "otc_multi_ctr_resident": (c_int, [c_int, P(c_vp), c_sz, K, c_u8p, c_int, P(ctypes.c_double)]),
        "otc_build_info": (ctypes.c_char_p, []),
        "otc_runtime_info": (c_int, [ctypes.c_char_p, c_sz]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def runtime_info() -> dict:
    """The HIP runtime / driver and RCCL versions this process runs on and the
    mapped libamdhip64 / librccl paths (otc_runtime_info): in a torch process
    the library binds torch's bundled HIP 7.0 and RCCL, in otbench and the
    CLIs /opt/rocm's 7.2 -- every A/B record names which."""
    import json

    lib = require_gpu_lib()
    buf = ctypes.create_string_buffer(4096)
    check(lib.otc_runtime_info(buf, len(buf)), "otc_runtime_info")
    return json.loads(buf.value.decode())


def gpu_lib_available() -> bool:
    return os.path.exists(GPU_LIB_PATH)


def require_gpu_lib():
    """Load libotc.so (HIP kernels).  Raises if it has not been built: device
    ops never fall back to Python/PyTorch silently."""
    global _gpu_lib
    if _gpu_lib is not None:
        return _gpu_lib
    with _lock:
        if _gpu_lib is None:
            if not os.path.exists(GPU_LIB_PATH):
                raise RuntimeError(
                    f"native HIP library missing: {GPU_LIB_PATH}; run `make` (or __graft_entry__.build())"
                )
            try:  # bind to torch's HIP runtime first, if torch is importable
                import torch  # noqa: F401
            except Exception:
                pass
            lib = ctypes.CDLL(GPU_LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            _declare_gpu(lib)
            _gpu_lib = lib
            atexit.register(_release_at_exit)
    return _gpu_lib


def _release_at_exit():
    """Return the library's pooled device objects (the split's auxiliary
    streams, the multi-GPU job's RCCL communicators) while the HIP runtime is
    still up: left to the runtime's own teardown, the CU-masked auxiliary
    streams were destroyed after a profiler's finalisation had run, and
    ``rocprofv3`` then crashed in ``__cxa_finalize`` at the process's exit
    (profiles/r6/rocprof/bench_full_exit_segv.txt)."""
    if _gpu_lib is not None:
        try:
            _gpu_lib.otc_release_resources()
        except Exception:  # noqa: BLE001 -- best effort at interpreter exit
            pass


def cpu_lib():
    """CPU oracle (reference-compatible C API).  Uses libotc_cpu.so so CPU-only
    tests never touch ROCm."""
    global _cpu_lib
    if _cpu_lib is not None:
        return _cpu_lib
    with _lock:
        if _cpu_lib is None:
            path = CPU_LIB_PATH if os.path.exists(CPU_LIB_PATH) else GPU_LIB_PATH
            if not os.path.exists(path):
                raise RuntimeError(f"native library missing: {CPU_LIB_PATH}; run `make cpu`")
            lib = ctypes.CDLL(path)
            _declare_cpu(lib)
            _cpu_lib = lib
    return _cpu_lib


def check(rc: int, what: str = "otc call"):
    if rc != 0:
        msg = require_gpu_lib().otc_last_error()
        raise RuntimeError(f"{what} failed (rc={rc}): {msg.decode() if msg else ''}")


def as_u8p(buf) -> ctypes.POINTER(ctypes.c_uint8):
    """bytes/bytearray/numpy/ctypes array -> uint8* (bytes are copied into a
    writable buffer by the caller when mutation is expected)."""
    if isinstance(buf, (bytes,)):
        return ctypes.cast(ctypes.c_char_p(buf), c_u8p)
    if isinstance(buf, bytearray):
        return (ctypes.c_uint8 * len(buf)).from_buffer(buf)
    try:
        import numpy as np

        if isinstance(buf, np.ndarray):
            return buf.ctypes.data_as(c_u8p)
    except Exception:
        pass
    return ctypes.cast(buf, c_u8p)
