"""Byte-stream device ops: XOR combiner (device ``arc4_crypt``), many-stream
RC4, synthetic fill and checksum -- kernels in ``csrc/hip/stream_ops.hip``."""
from __future__ import annotations

import ctypes

import torch

from .. import _native
from .aes_ops import _bytes, _check_dev, _nbytes, _run, _stream


def xor(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """out = a ^ b (bytewise).  Reference arc4_crypt (arc4.c:101-112) on the GPU."""
    _check_dev(a, "a")
    _check_dev(b, "b")
    if _nbytes(a) != _nbytes(b):
        raise ValueError("a and b must have the same byte size")
    out = torch.empty_like(a) if out is None else out
    if b.data_ptr() % 16:
        b = _bytes(b).clone()  # 16-byte alignment (a and out are staged by _run)
    with torch.cuda.device(a.device):
        rc = _run(a, out, lambda ip, op: _native.require_gpu_lib().otc_xor(
            ip, b.data_ptr(), op, _nbytes(a), _stream(a)))
    _native.check(rc, "otc_xor")
    return out


def rc4_multi(keys: torch.Tensor, length: int, x: torch.Tensor | None = None, drop: int = 0,
              out: torch.Tensor | None = None) -> torch.Tensor:
    """Run ``keys.shape[0]`` independent RC4 streams (one per GPU lane).

    keys: uint8 [nstreams, keylen] on the GPU.  Returns uint8 [nstreams, length]:
    the keystream, or ``x ^ keystream`` when ``x`` (same shape) is given."""
    _check_dev(keys, "keys")
    if keys.dtype != torch.uint8 or keys.dim() != 2:
        raise ValueError("keys must be uint8 [nstreams, keylen]")
    ns, kl = keys.shape
    if x is not None:
        _check_dev(x, "x")
        if _nbytes(x) != ns * length:
            raise ValueError("x must hold nstreams*length bytes")
    out = torch.empty((ns, length), dtype=torch.uint8, device=keys.device) if out is None else out
    with torch.cuda.device(keys.device):
        rc = _native.require_gpu_lib().otc_rc4_multi(keys.data_ptr(), kl, ns, length, drop,
                                                     x.data_ptr() if x is not None else None, out.data_ptr(),
                                                     _stream(keys))
    _native.check(rc, "otc_rc4_multi")
    return out


RC4_STATE_BYTES = 264  # sizeof(struct rc4_state): char perm[256]; int index1, index2


def rc4_states(keys) -> torch.Tensor:
    """``rc4_init`` (rc4.h) of every key on the host: uint8 [n, 264] CPU
    tensor of ``struct rc4_state`` images, ready to move to the GPU."""
    lib = _native.cpu_lib()
    out = torch.empty((len(keys), RC4_STATE_BYTES), dtype=torch.uint8)
    for r, k in enumerate(keys):
        st = _native.Rc4State()
        k = bytes(k)
        lib.rc4_init(ctypes.byref(st), k, len(k))
        out[r] = torch.frombuffer(bytearray(bytes(st)), dtype=torch.uint8)
    return out


def rc4_crypt_batch(states: torch.Tensor, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """``rc4_crypt`` (rc4.h) for many streams on the GPU: ``states`` uint8
    [n, 264] device tensor of ``struct rc4_state`` (see :func:`rc4_states`),
    ``x`` [n, len] bytes; returns x ^ keystream and advances every state in
    place, so a later call resumes each stream exactly where it stopped."""
    _check_dev(states, "states")
    _check_dev(x, "x")
    if states.dtype != torch.uint8 or states.dim() != 2 or states.shape[1] != RC4_STATE_BYTES:
        raise ValueError(f"states must be uint8 [nstreams, {RC4_STATE_BYTES}]")
    ns = states.shape[0]
    if ns == 0 or _nbytes(x) % ns:
        raise ValueError("x must hold nstreams * len bytes")
    length = _nbytes(x) // ns
    out = torch.empty_like(x) if out is None else out
    _check_dev(out, "out")
    if _nbytes(out) != _nbytes(x):
        raise ValueError("out must have the byte size of x")
    if not (states.device == x.device == out.device):
        raise ValueError(f"states, x and out must be on one device (got {states.device}, {x.device}, {out.device})")
    with torch.cuda.device(x.device):
        rc = _native.require_gpu_lib().otc_rc4_crypt_batch(states.data_ptr(), ns, length, x.data_ptr(),
                                                           out.data_ptr(), _stream(x))
    _native.check(rc, "otc_rc4_crypt_batch")
    return out


def fill_random_(t: torch.Tensor, seed: int = 0) -> torch.Tensor:
    """Fill ``t`` in place with deterministic pseudo-random bytes (splitmix64)."""
    _check_dev(t, "t")
    with torch.cuda.device(t.device):
        rc = _run(t, t, lambda ip, op: _native.require_gpu_lib().otc_fill_random(
            op, _nbytes(t), seed & (2**64 - 1), _stream(t)))
    _native.check(rc, "otc_fill_random")
    return t


def checksum(t: torch.Tensor) -> int:
    """Position-dependent 64-bit XOR fold of a device buffer (byte size % 8 == 0)."""
    _check_dev(t, "t")
    acc = torch.zeros(1, dtype=torch.int64, device=t.device)
    if t.data_ptr() % 8:
        t = _bytes(t).clone()  # the fold reads 8-byte words
    with torch.cuda.device(t.device):
        rc = _native.require_gpu_lib().otc_checksum(t.data_ptr(), _nbytes(t), acc.data_ptr(), _stream(t))
    _native.check(rc, "otc_checksum")
    return int(acc.item()) & (2**64 - 1)


def clock_probe(delay_s: float, window_s: float, device=None, stream=None) -> torch.Tensor:
    """Launch the one-wave clock probe (``otc_clock_probe``) on ``stream``
    (default: a new side stream) and return its 2-element result tensor; read
    it with :func:`clock_ghz` after the workload has been synchronized."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    out = torch.zeros(2, dtype=torch.int64, device=dev)
    s = stream if stream is not None else torch.cuda.Stream(device=dev)
    with torch.cuda.device(dev):
        rc = _native.require_gpu_lib().otc_clock_probe(out.data_ptr(), float(delay_s), float(window_s),
                                                       ctypes.c_void_p(s.cuda_stream))
    _native.check(rc, "otc_clock_probe")
    out._probe_stream = s  # keep the side stream alive until the result is read
    return out


def clock_ghz(probe: torch.Tensor) -> float:
    cyc, ticks = (int(v) for v in probe.cpu().tolist())
    return 0.1 * cyc / ticks if ticks > 0 else float("nan")
