"""AES key expansion for the device kernels (round keys travel BY VALUE as a
kernel argument, i.e. in SGPRs -- no per-call device copy; contrast the
reference's per-makeKey cudaMemcpy, /root/reference/aes-gpu/Source/AES.cu:205-228)."""
from __future__ import annotations

import ctypes
import functools

from .. import _native

ENCRYPT = 1
DECRYPT = 0


@functools.lru_cache(maxsize=256)
def _expand(key: bytes, direction: int) -> _native.OtcAesKey:
    bits = len(key) * 8
    if bits not in (128, 192, 256):
        raise ValueError(f"AES key must be 16/24/32 bytes, got {len(key)}")
    k = _native.OtcAesKey()
    rc = _native.require_gpu_lib().otc_aes_key_init(ctypes.byref(k), _native.as_u8p(key), bits, direction)
    _native.check(rc, "otc_aes_key_init")
    return k


def expand_key(key: bytes, decrypt: bool = False) -> _native.OtcAesKey:
    """Return the cached ``otc_aes_key`` for ``key`` (encryption or equivalent
    inverse-cipher schedule)."""
    return _expand(bytes(key), DECRYPT if decrypt else ENCRYPT)
