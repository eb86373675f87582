"""The AES "model family": a BlockCipher-style object over the gfx950 kernels.

Parity: the reference's ``BlockCipher`` interface and ``AES`` host class
(/root/reference/aes-gpu/Source/BlockCipher.h:48-107, AES.h:84-147):
block/key size queries, ``make_key(key, bits, direction)``, ``encrypt`` /
``decrypt`` of n blocks -- extended with every mode the CPU API offers
(CBC, CFB128, CTR) plus sharding-friendly counter offsets.  GPU tensors go to
the HIP kernels; ``bytes`` go to the C oracle.
"""
from __future__ import annotations

import torch

from .. import ops
from . import cpu_ref

DIR_NONE, DIR_ENCRYPT, DIR_DECRYPT = 0, 1, 2
DIR_BOTH = DIR_ENCRYPT | DIR_DECRYPT


class AES:
    block_bits = 128
    block_size = 16

    def __init__(self, key: bytes | None = None, impl: str = "auto"):
        self._key = None
        self.impl = impl
        if key is not None:
            self.make_key(key)

    # ---- BlockCipher interface -------------------------------------------
    def make_key(self, key: bytes, key_bits: int | None = None, direction: int = DIR_BOTH):
        key = bytes(key)
        if key_bits is not None and key_bits != len(key) * 8:
            raise ValueError("key_bits does not match the key length")
        if len(key) not in (16, 24, 32):
            raise ValueError("Invalid AES key size.")
        self._key = key
        if direction & DIR_ENCRYPT:
            ops.expand_key(key)
        if direction & DIR_DECRYPT:
            ops.expand_key(key, decrypt=True)
        return self

    @property
    def key_bits(self) -> int:
        return len(self._key) * 8

    @property
    def key_size(self) -> int:
        return len(self._key)

    @property
    def rounds(self) -> int:
        return {16: 10, 24: 12, 32: 14}[len(self._key)]

    def encrypt(self, data, out=None):
        """ECB encryption of whole blocks."""
        if isinstance(data, torch.Tensor):
            return ops.ecb_encrypt(data, self._key, out=out, impl=self.impl)
        return cpu_ref.ecb(self._key, data)

    def decrypt(self, data, out=None):
        if isinstance(data, torch.Tensor):
            return ops.ecb_decrypt(data, self._key, out=out, impl=self.impl)
        return cpu_ref.ecb(self._key, data, decrypt=True)

    # ---- modes -------------------------------------------------------------
    def ctr(self, data, counter: bytes, block_offset: int = 0, out=None):
        if isinstance(data, torch.Tensor):
            return ops.ctr(data, self._key, counter, out=out, block_offset=block_offset, impl=self.impl)
        return cpu_ref.ctr(self._key, counter, data, block_offset)

    # exact single-stream CBC / CFB encryption is one serial chain: on a GPU it
    # would run on ONE lane (~67M dependent block encryptions per GiB), far
    # slower than one AES-NI core, so GPU tensors take the host chain unless
    # the caller opts in with device_serial=True (small buffers, no host trip)
    def _serial_on_host(self, mode: str, data: torch.Tensor, iv: bytes, out):
        res = cpu_ref.serial_encrypt(mode, self._key, iv, data.reshape(-1).view(torch.uint8).cpu().numpy().tobytes())
        t = torch.frombuffer(bytearray(res), dtype=torch.uint8).to(data.device)
        if out is None:
            return t.view(data.dtype).view(data.shape)
        out.reshape(-1).view(torch.uint8).copy_(t)
        return out

    def cbc_encrypt(self, data, iv: bytes, segment_bytes: int | None = None, out=None, device_serial: bool = False):
        """CBC encryption.  ``segment_bytes``: independent segments with
        IV_s = iv + s (parallel, one lane per segment); None = one exact
        serial stream (host AES-NI chain for GPU tensors, see above)."""
        if isinstance(data, torch.Tensor):
            if segment_bytes:
                return ops.cbc_encrypt_segments(data, self._key, iv, segment_bytes, out=out)
            if device_serial:
                return ops.cbc_encrypt_segments(data, self._key, iv, data.numel() * data.element_size(), out=out)
            return self._serial_on_host("cbc", data, iv, out)
        if segment_bytes:
            return cpu_ref.cbc_segments(self._key, iv, data, segment_bytes)
        return cpu_ref.serial_encrypt("cbc", self._key, iv, data)

    def cbc_decrypt(self, data, iv: bytes, segment_bytes: int | None = None, out=None):
        if isinstance(data, torch.Tensor):
            if segment_bytes:
                return ops.cbc_decrypt_segments(data, self._key, iv, segment_bytes, out=out)
            return ops.cbc_decrypt(data, self._key, iv, out=out, impl=self.impl)
        if segment_bytes:
            return cpu_ref.cbc_segments(self._key, iv, data, segment_bytes, decrypt=True)
        return cpu_ref.cbc(self._key, iv, data, decrypt=True)

    def cfb128_decrypt(self, data, iv: bytes, segment_bytes: int | None = None, out=None):
        if isinstance(data, torch.Tensor):
            if segment_bytes:
                return ops.cfb128_decrypt_segments(data, self._key, iv, segment_bytes, out=out)
            return ops.cfb128_decrypt(data, self._key, iv, out=out, impl=self.impl)
        if segment_bytes:
            return cpu_ref.cfb128_segments(self._key, iv, data, segment_bytes, decrypt=True)
        return cpu_ref.cfb128(self._key, iv, data, decrypt=True)

    def cfb128_encrypt(self, data, iv: bytes, segment_bytes: int | None = None, out=None,
                       device_serial: bool = False):
        """CFB128 encryption (reference aes-modes/aes.c:822-862): a serial
        chain.  ``segment_bytes``: independent segments with IV_s = iv + s on
        the GPU sector kernel; None = exact single stream (host AES-NI chain
        for GPU tensors unless ``device_serial``)."""
        if isinstance(data, torch.Tensor):
            if segment_bytes:
                return ops.cfb128_encrypt_segments(data, self._key, iv, segment_bytes, out=out)
            if device_serial:
                return ops.cfb128_encrypt_segments(data, self._key, iv, data.numel() * data.element_size(), out=out)
            return self._serial_on_host("cfb128", data, iv, out)
        if segment_bytes:
            return cpu_ref.cfb128_segments(self._key, iv, data, segment_bytes)
        return cpu_ref.serial_encrypt("cfb128", self._key, iv, data)
