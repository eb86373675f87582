"""Device AES ops on torch tensors (ROCm ``cuda`` tensors), backed by the
hand-written gfx950 kernels in ``csrc/hip/aes_tt.hip`` (LDS T-table) and
``csrc/hip/aes_bs.hip`` (bitsliced VALU).

Every op runs asynchronously on torch's current HIP stream and raises on any
native error.  Tensors may have any dtype; they are treated as contiguous byte
buffers.  Reference kernels: /root/reference/aes-gpu/Source/AES.cu:284-502
(ECB only, broken launch); everything else here is new capability.
"""
from __future__ import annotations

import ctypes

import torch

from .. import _native
from .keys import expand_key

IMPLS = {"auto": 0, "ttable": 1, "bitslice": 2, "hybrid": 3}


def _impl(impl) -> int:
    if isinstance(impl, int):
        return impl
    try:
        return IMPLS[impl]
    except KeyError:
        raise ValueError(f"impl must be one of {list(IMPLS)}") from None


def _check_dev(t: torch.Tensor, name: str):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise ValueError(f"{name} must be a GPU tensor (got {t.device})")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def _nbytes(t: torch.Tensor) -> int:
    return t.numel() * t.element_size()


def _stream(t: torch.Tensor):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _out_like(x: torch.Tensor, out):
    if out is None:
        return torch.empty_like(x)
    _check_dev(out, "out")
    if _nbytes(out) != _nbytes(x):
        raise ValueError("out must have the same byte size as the input")
    return out


def _bytes(t: torch.Tensor) -> torch.Tensor:
    """Flat uint8 view of a contiguous tensor."""
    return t.reshape(-1).view(torch.uint8)


def _run(x: torch.Tensor, out: torch.Tensor, call):
    """call(in_ptr, out_ptr) -> rc.  The kernels move 16 bytes per lane, so the
    native API requires 16-byte aligned buffers; a misaligned tensor (e.g. a
    byte slice ``t[3:]``) is staged through an aligned temporary (torch's
    allocator aligns every fresh allocation) and copied back."""
    xp, op = x.data_ptr(), out.data_ptr()
    if not (xp % 16 or op % 16) or _nbytes(x) == 0:
        return call(xp, op)
    xi = _bytes(x).clone() if xp % 16 else _bytes(x)
    if op == xp:
        xo = xi  # in place stays in place (the native API rejects modes that forbid it)
    elif op % 16:
        xo = torch.empty_like(xi)
    else:
        xo = _bytes(out)
    rc = call(xi.data_ptr(), xo.data_ptr())
    if rc == 0 and xo.data_ptr() != op:
        _bytes(out).copy_(xo)
    return rc


def _b16(v, name) -> ctypes.Array:
    v = bytes(v)
    if len(v) != 16:
        raise ValueError(f"{name} must be 16 bytes")
    return (ctypes.c_uint8 * 16).from_buffer_copy(v)


def _lib():
    return _native.require_gpu_lib()


def ctr(x: torch.Tensor, key: bytes, counter: bytes, out: torch.Tensor | None = None, block_offset: int = 0,
        impl="auto") -> torch.Tensor:
    """AES-CTR (128-bit big-endian counter starting at ``counter`` + ``block_offset``)."""
    _check_dev(x, "x")
    out = _out_like(x, out)
    k = expand_key(key)
    with torch.cuda.device(x.device):
        rc = _run(x, out, lambda ip, op: _lib().otc_aes_ctr(ip, op, _nbytes(x), ctypes.byref(k), _b16(counter, "counter"),
            int(block_offset), _impl(impl), _stream(x)))
    _native.check(rc, "otc_aes_ctr")
    return out


def ctr_rfc3686(x: torch.Tensor, key: bytes, nonce: bytes, ivec: bytes, out=None, block_offset: int = 0,
                impl="auto") -> torch.Tensor:
    """AES-CTR with the AES-NI/RFC 3686 counter block nonce||ivec||BE32(1) and
    64-bit increment (reference aesni.c:120-152)."""
    _check_dev(x, "x")
    out = _out_like(x, out)
    k = expand_key(key)
    n = (ctypes.c_uint8 * 4).from_buffer_copy(bytes(nonce))
    iv = (ctypes.c_uint8 * 8).from_buffer_copy(bytes(ivec))
    with torch.cuda.device(x.device):
        rc = _run(x, out, lambda ip, op: _lib().otc_aes_ctr_rfc3686(ip, op, _nbytes(x), ctypes.byref(k), n, iv,
            int(block_offset), _impl(impl), _stream(x)))
    _native.check(rc, "otc_aes_ctr_rfc3686")
    return out


def ecb_encrypt(x: torch.Tensor, key: bytes, out=None, impl="auto") -> torch.Tensor:
    _check_dev(x, "x")
    out = _out_like(x, out)
    k = expand_key(key)
    with torch.cuda.device(x.device):
        rc = _run(x, out, lambda ip, op: _lib().otc_aes_ecb(ip, op, _nbytes(x), ctypes.byref(k), _impl(impl), _stream(x)))
    _native.check(rc, "otc_aes_ecb(encrypt)")
    return out


def ecb_decrypt(x: torch.Tensor, key: bytes, out=None) -> torch.Tensor:
    _check_dev(x, "x")
    out = _out_like(x, out)
    k = expand_key(key, decrypt=True)
    with torch.cuda.device(x.device):
        rc = _run(x, out, lambda ip, op: _lib().otc_aes_ecb(ip, op, _nbytes(x), ctypes.byref(k), 0, _stream(x)))
    _native.check(rc, "otc_aes_ecb(decrypt)")
    return out


def cbc_decrypt(x: torch.Tensor, key: bytes, iv: bytes, out=None) -> torch.Tensor:
    """Parallel CBC decryption (out must not alias x)."""
    _check_dev(x, "x")
    out = _out_like(x, out)
    k = expand_key(key, decrypt=True)
    with torch.cuda.device(x.device):
        rc = _run(x, out, lambda ip, op: _lib().otc_aes_cbc_decrypt(ip, op, _nbytes(x), ctypes.byref(k), _b16(iv, "iv"),
            _stream(x)))
    _native.check(rc, "otc_aes_cbc_decrypt")
    return out


def cbc_encrypt_segments(x: torch.Tensor, key: bytes, iv0: bytes, segment_bytes: int, out=None) -> torch.Tensor:
    """CBC encryption of independent contiguous segments; segment s uses
    IV = iv0 + s (128-bit BE).  One segment == exact serial CBC."""
    _check_dev(x, "x")
    out = _out_like(x, out)
    n = _nbytes(x)
    if segment_bytes <= 0 or n % segment_bytes:
        raise ValueError("byte size must be a multiple of segment_bytes")
    k = expand_key(key)
    with torch.cuda.device(x.device):
        rc = _run(x, out, lambda ip, op: _lib().otc_aes_cbc_encrypt_segments(ip, op, segment_bytes, n // segment_bytes,
            ctypes.byref(k), _b16(iv0, "iv0"), _stream(x)))
    _native.check(rc, "otc_aes_cbc_encrypt_segments")
    return out


def cbc_decrypt_segments(x: torch.Tensor, key: bytes, iv0: bytes, segment_bytes: int, out=None) -> torch.Tensor:
    _check_dev(x, "x")
    out = _out_like(x, out)
    n = _nbytes(x)
    if segment_bytes <= 0 or n % segment_bytes:
        raise ValueError("byte size must be a multiple of segment_bytes")
    k = expand_key(key, decrypt=True)
    with torch.cuda.device(x.device):
        rc = _run(x, out, lambda ip, op: _lib().otc_aes_cbc_decrypt_segments(ip, op, segment_bytes, n // segment_bytes,
            ctypes.byref(k), _b16(iv0, "iv0"), _stream(x)))
    _native.check(rc, "otc_aes_cbc_decrypt_segments")
    return out


def cfb128_decrypt(x: torch.Tensor, key: bytes, iv: bytes, out=None) -> torch.Tensor:
    _check_dev(x, "x")
    out = _out_like(x, out)
    k = expand_key(key)
    with torch.cuda.device(x.device):
        rc = _run(x, out, lambda ip, op: _lib().otc_aes_cfb128_decrypt(ip, op, _nbytes(x), ctypes.byref(k), _b16(iv, "iv"),
            _stream(x)))
    _native.check(rc, "otc_aes_cfb128_decrypt")
    return out
