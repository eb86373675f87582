"""Cipher "model families": AES (ECB/CBC/CFB128/CTR, 128/192/256) and ARC4/RC4."""
from . import cpu_ref
from .aes import AES, DIR_BOTH, DIR_DECRYPT, DIR_ENCRYPT, DIR_NONE
from .arc4 import ARC4, RC4MultiStream

__all__ = ["AES", "ARC4", "RC4MultiStream", "cpu_ref", "DIR_NONE", "DIR_ENCRYPT", "DIR_DECRYPT", "DIR_BOTH"]
