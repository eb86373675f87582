"""The ARC4/RC4 "model family".

``ARC4`` keeps the reference's producer/consumer split (serial keystream
``arc4_prep`` on the CPU, parallel ``arc4_crypt`` XOR -- here on the GPU), see
/root/reference/test.c:60-126 and arc4.c:72-112.  ``RC4MultiStream`` is the
GPU-native design: thousands of independent keys, one RC4 state per lane in
LDS (csrc/hip/stream_ops.hip).
"""
from __future__ import annotations

import torch

from .. import ops
from . import cpu_ref


class ARC4:
    def __init__(self, key: bytes):
        self.key = bytes(key)
        self._drop = 0

    def keystream(self, n: int) -> bytes:
        """Next ``n`` keystream bytes (resumable, like arc4_prep)."""
        ks = cpu_ref.arc4_keystream(self.key, n, drop=self._drop)
        self._drop += n
        return ks

    def crypt(self, data, keystream=None):
        """XOR ``data`` with the keystream.  GPU tensors use the device combiner."""
        if isinstance(data, torch.Tensor):
            n = data.numel() * data.element_size()
            if keystream is None:
                keystream = self.keystream(n)
            if not isinstance(keystream, torch.Tensor):
                keystream = torch.frombuffer(bytearray(keystream), dtype=torch.uint8).to(data.device)
            return ops.xor(data.view(torch.uint8).reshape(-1), keystream.reshape(-1)).view_as(data)
        if keystream is None:
            keystream = self.keystream(len(data))
        return cpu_ref.arc4_crypt(data, keystream)


class RC4MultiStream:
    """Many independent RC4 streams on the GPU (keys: uint8 [n, keylen])."""

    def __init__(self, keys: torch.Tensor, drop: int = 0):
        self.keys = keys
        self.drop = drop

    def keystream(self, length: int) -> torch.Tensor:
        return ops.rc4_multi(self.keys, length, drop=self.drop)

    def crypt(self, x: torch.Tensor) -> torch.Tensor:
        return ops.rc4_multi(self.keys, x.shape[-1], x=x, drop=self.drop)
