"""CPU oracle wrappers (bytes in, bytes out) over the C reference-compatible
API in ``csrc/cpu`` (aes.h / arc4.h / rc4.h / aesni.h).  Used by the tests, by
the CPU fallback of the distributed planner tests, and as the verification
oracle for every device kernel.  API parity: /root/reference/aes-modes/aes.h,
/root/reference/arc4.h, /root/reference/rc4.h, /root/reference/aes-modes/aesni.h.
"""
from __future__ import annotations

import ctypes

from .. import _native

AES_ENCRYPT = 1
AES_DECRYPT = 0


def _ctx(key: bytes, decrypt: bool = False) -> _native.AesContext:
    lib = _native.cpu_lib()
    ctx = _native.AesContext()
    fn = lib.aes_setkey_dec if decrypt else lib.aes_setkey_enc
    rc = fn(ctypes.byref(ctx), _native.as_u8p(bytes(key)), len(key) * 8)
    if rc:
        raise ValueError("invalid AES key length")
    return ctx


def _buf(n: int):
    return (ctypes.c_uint8 * max(n, 1))()


def ecb(key: bytes, data: bytes, decrypt: bool = False, threads: int = 1) -> bytes:
    if len(data) % 16:
        raise ValueError("ECB needs a multiple of 16 bytes")
    ctx = _ctx(key, decrypt)
    out = _buf(len(data))
    _native.cpu_lib().aes_ecb_bulk(ctypes.byref(ctx), AES_DECRYPT if decrypt else AES_ENCRYPT,
                                   _native.as_u8p(bytes(data)), out, len(data), threads)
    return bytes(out)[: len(data)]


def ctr(key: bytes, counter: bytes, data: bytes, block_offset: int = 0, threads: int = 1) -> bytes:
    ctx = _ctx(key)
    nc = (ctypes.c_uint8 * 16).from_buffer_copy(bytes(counter))
    if block_offset:
        _native.cpu_lib().aes_ctr128_add(nc, block_offset)
    out = _buf(len(data))
    _native.cpu_lib().aes_ctr_bulk(ctypes.byref(ctx), nc, _native.as_u8p(bytes(data)), out, len(data), threads)
    return bytes(out)[: len(data)]


def ctr_stream(key: bytes, nonce_counter: bytearray, stream_block: bytearray, nc_off: list, data: bytes) -> bytes:
    """Byte-granular resumable CTR exactly as aes_crypt_ctr (updates the
    counter, stream block and offset in place)."""
    ctx = _ctx(key)
    nc = (ctypes.c_uint8 * 16).from_buffer(nonce_counter)
    sb = (ctypes.c_uint8 * 16).from_buffer(stream_block)
    off = ctypes.c_int(nc_off[0])
    out = _buf(len(data))
    _native.cpu_lib().aes_crypt_ctr(ctypes.byref(ctx), len(data), ctypes.byref(off), nc, sb,
                                    _native.as_u8p(bytes(data)), out)
    nc_off[0] = off.value
    return bytes(out)[: len(data)]


def cbc(key: bytes, iv: bytes, data: bytes, decrypt: bool = False) -> bytes:
    ctx = _ctx(key, decrypt)
    ivb = (ctypes.c_uint8 * 16).from_buffer_copy(bytes(iv))
    out = _buf(len(data))
    rc = _native.cpu_lib().aes_crypt_cbc(ctypes.byref(ctx), AES_DECRYPT if decrypt else AES_ENCRYPT, len(data), ivb,
                                         _native.as_u8p(bytes(data)), out)
    if rc:
        raise ValueError("CBC needs a multiple of 16 bytes")
    return bytes(out)[: len(data)]


def cfb128(key: bytes, iv: bytes, data: bytes, decrypt: bool = False) -> bytes:
    ctx = _ctx(key)
    ivb = (ctypes.c_uint8 * 16).from_buffer_copy(bytes(iv))
    off = ctypes.c_int(0)
    out = _buf(len(data))
    _native.cpu_lib().aes_crypt_cfb128(ctypes.byref(ctx), AES_DECRYPT if decrypt else AES_ENCRYPT, len(data),
                                       ctypes.byref(off), ivb, _native.as_u8p(bytes(data)), out)
    return bytes(out)[: len(data)]


def ctr128_add(counter: bytes, blocks: int) -> bytes:
    v = (int.from_bytes(bytes(counter), "big") + blocks) % (1 << 128)
    return v.to_bytes(16, "big")


def cbc_segments(key: bytes, iv0: bytes, data: bytes, segment_bytes: int, decrypt: bool = False) -> bytes:
    """Per-segment CBC with IV_s = iv0 + s (the device segment semantics)."""
    out = bytearray()
    for s, off in enumerate(range(0, len(data), segment_bytes)):
        out += cbc(key, ctr128_add(iv0, s), data[off: off + segment_bytes], decrypt)
    return bytes(out)


def cfb128_segments(key: bytes, iv0: bytes, data: bytes, segment_bytes: int, decrypt: bool = False) -> bytes:
    """Per-segment CFB128 with IV_s = iv0 + s (the device segment semantics)."""
    out = bytearray()
    for s, off in enumerate(range(0, len(data), segment_bytes)):
        out += cfb128(key, ctr128_add(iv0, s), data[off: off + segment_bytes], decrypt)
    return bytes(out)


def serial_encrypt(mode: str, key: bytes, iv: bytes, data: bytes) -> bytes:
    """Exact single-stream CBC / CFB128 encryption on one core with AES-NI
    (the C oracle where AES-NI is absent).  This is the host path for the
    serial chain: a GPU runs it on one lane, far slower than one x86 core."""
    if mode not in ("cbc", "cfb128"):
        raise ValueError("mode must be 'cbc' or 'cfb128'")
    if mode == "cbc" and len(data) % 16:
        raise ValueError("CBC needs a multiple of 16 bytes")
    if not aesni_supported():
        return cbc(key, iv, data) if mode == "cbc" else cfb128(key, iv, data)
    sched, nr = aesni_schedule(key)
    ivb = (ctypes.c_uint8 * 16).from_buffer_copy(bytes(iv))
    out = _buf(len(data))
    fn = _native.cpu_lib().AES_CBC_encrypt if mode == "cbc" else _native.cpu_lib().AES_CFB128_encrypt
    fn(_native.as_u8p(bytes(data)), out, ivb, len(data), _native.as_u8p(sched), nr)
    return bytes(out)[: len(data)]


def arc4_keystream(key: bytes, n: int, drop: int = 0) -> bytes:
    lib = _native.cpu_lib()
    ctx = _native.Arc4Context()
    lib.arc4_setup(ctypes.byref(ctx), _native.as_u8p(bytes(key)), len(key))
    if drop:
        lib.arc4_prep(ctypes.byref(ctx), drop, _buf(drop))
    ks = _buf(n)
    lib.arc4_prep(ctypes.byref(ctx), n, ks)
    return bytes(ks)[:n]


def arc4_crypt(data: bytes, keystream: bytes, threads: int = 1) -> bytes:
    out = _buf(len(data))
    _native.cpu_lib().arc4_crypt_mt(len(data), _native.as_u8p(bytes(data)), _native.as_u8p(bytes(keystream)), out,
                                    threads)
    return bytes(out)[: len(data)]


def rc4_oneshot(key: bytes, data: bytes) -> bytes:
    """rc4.h API (rc4_init + rc4_crypt)."""
    lib = _native.cpu_lib()
    st = _native.Rc4State()
    lib.rc4_init(ctypes.byref(st), bytes(key), len(key))
    out = ctypes.create_string_buffer(max(len(data), 1))
    lib.rc4_crypt(ctypes.byref(st), bytes(data), out, len(data))
    return out.raw[: len(data)]


def aesni_supported() -> bool:
    return bool(_native.cpu_lib().CheckAESSupport())


def aesni_ctr(key: bytes, nonce: bytes, ivec: bytes, data: bytes, block_offset: int = 0) -> bytes:
    lib = _native.cpu_lib()
    nr = {16: 10, 24: 12, 32: 14}[len(key)]
    sched = (ctypes.c_uint8 * 240)()
    {10: lib.AES_128_Key_Expansion, 12: lib.AES_192_Key_Expansion, 14: lib.AES_256_Key_Expansion}[nr](
        _native.as_u8p(bytes(key)), sched)
    out = _buf(len(data))
    lib.AES_CTR_encrypt_at(_native.as_u8p(bytes(data)), out, _native.as_u8p(bytes(ivec)), _native.as_u8p(bytes(nonce)),
                           len(data), sched, nr, block_offset)
    return bytes(out)[: len(data)]


def aesni_schedule(key: bytes, decrypt: bool = False):
    """(schedule bytes, Nr) as AES_*_Key_Expansion / AES_Key_Expansion_Dec
    produce them (16*(Nr+1) bytes)."""
    lib = _native.cpu_lib()
    nr = {16: 10, 24: 12, 32: 14}[len(key)]
    sched = (ctypes.c_uint8 * 240)()
    {10: lib.AES_128_Key_Expansion, 12: lib.AES_192_Key_Expansion, 14: lib.AES_256_Key_Expansion}[nr](
        _native.as_u8p(bytes(key)), sched)
    if decrypt:
        dsched = (ctypes.c_uint8 * 240)()
        lib.AES_Key_Expansion_Dec(sched, dsched, nr)
        sched = dsched
    return bytes(sched)[: 16 * (nr + 1)], nr


def aesni_ecb(key: bytes, data: bytes, decrypt: bool = False) -> bytes:
    lib = _native.cpu_lib()
    nr = {16: 10, 24: 12, 32: 14}[len(key)]
    sched = (ctypes.c_uint8 * 240)()
    {10: lib.AES_128_Key_Expansion, 12: lib.AES_192_Key_Expansion, 14: lib.AES_256_Key_Expansion}[nr](
        _native.as_u8p(bytes(key)), sched)
    out = _buf(len(data))
    if decrypt:
        dsched = (ctypes.c_uint8 * 240)()
        lib.AES_Key_Expansion_Dec(sched, dsched, nr)
        lib.AES_ECB_decrypt(_native.as_u8p(bytes(data)), out, len(data), dsched, nr)
    else:
        lib.AES_ECB_encrypt(_native.as_u8p(bytes(data)), out, len(data), sched, nr)
    return bytes(out)[: len(data)]


def self_tests(verbose: int = 0) -> dict:
    lib = _native.cpu_lib()
    return {
        "aes": lib.aes_self_test(verbose),
        "arc4": lib.arc4_self_test(verbose),
        "bitslice": lib.otc_bitslice_selftest(verbose),
    }
