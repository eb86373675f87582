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
            return ops.ecb_decrypt(data, self._key, out=out)
        return cpu_ref.ecb(self._key, data, decrypt=True)

    # ---- modes -------------------------------------------------------------
    def ctr(self, data, counter: bytes, block_offset: int = 0, out=None):
        if isinstance(data, torch.Tensor):
            return ops.ctr(data, self._key, counter, out=out, block_offset=block_offset, impl=self.impl)
        return cpu_ref.ctr(self._key, counter, data, block_offset)

    def cbc_encrypt(self, data, iv: bytes, segment_bytes: int | None = None, out=None):
        """CBC encryption.  ``segment_bytes``: independent segments with
        IV_s = iv + s (parallel); None = one exact serial stream."""
        if isinstance(data, torch.Tensor):
            seg = segment_bytes or data.numel() * data.element_size()
            return ops.cbc_encrypt_segments(data, self._key, iv, seg, out=out)
        if segment_bytes:
            return cpu_ref.cbc_segments(self._key, iv, data, segment_bytes)
        return cpu_ref.cbc(self._key, iv, data)

    def cbc_decrypt(self, data, iv: bytes, segment_bytes: int | None = None, out=None):
        if isinstance(data, torch.Tensor):
            if segment_bytes:
                return ops.cbc_decrypt_segments(data, self._key, iv, segment_bytes, out=out)
            return ops.cbc_decrypt(data, self._key, iv, out=out)
        if segment_bytes:
            return cpu_ref.cbc_segments(self._key, iv, data, segment_bytes, decrypt=True)
        return cpu_ref.cbc(self._key, iv, data, decrypt=True)

    def cfb128_decrypt(self, data, iv: bytes, out=None):
        if isinstance(data, torch.Tensor):
            return ops.cfb128_decrypt(data, self._key, iv, out=out)
        return cpu_ref.cfb128(self._key, iv, data, decrypt=True)

    def cfb128_encrypt(self, data: bytes, iv: bytes):
        """CFB encryption is a serial chain -> CPU oracle only."""
        return cpu_ref.cfb128(self._key, iv, data)
