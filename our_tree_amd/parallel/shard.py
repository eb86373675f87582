"""Shard planner: byte ranges, CTR counter offsets and CBC halos.

Pure Python (no GPU) so the distribution logic is unit-tested on CPU
(SURVEY.md section 4, item 5 "fake multi-GPU").  The reference's only
"sharding" was pthread chunking that dropped the remainder
(/root/reference/test.c:44-58, aes-modes/test.c:28-44) and reused one CTR
keystream in every thread (aes-modes/test.c:282); here every shard is
block-aligned, the remainder is spread (nothing dropped) and each shard gets its
exact counter offset.
"""
from __future__ import annotations

from dataclasses import dataclass

BLOCK = 16


@dataclass(frozen=True)
class Shard:
    index: int
    offset: int        # byte offset in the global stream
    nbytes: int
    block_offset: int  # CTR: counter offset of the first byte (offset // 16)

    @property
    def end(self) -> int:
        return self.offset + self.nbytes

    @property
    def needs_halo(self) -> bool:
        """CBC decryption needs the ciphertext block preceding this shard."""
        return self.offset > 0


def plan(nbytes: int, nshards: int, align: int = BLOCK) -> list[Shard]:
    """Split ``nbytes`` into ``nshards`` contiguous ``align``-aligned shards;
    the first ``r`` shards take one extra unit.  The last shard also takes the
    trailing partial block (CTR)."""
    if nshards < 1:
        raise ValueError("nshards must be >= 1")
    if align % BLOCK:
        raise ValueError("align must be a multiple of 16")
    units = nbytes // align
    per, rem = divmod(units, nshards)
    out, off = [], 0
    for i in range(nshards):
        n = (per + (1 if i < rem else 0)) * align
        if i == nshards - 1:
            n = nbytes - off
        out.append(Shard(i, off, n, off // BLOCK))
        off += n
    return out


def equal_plan(nbytes: int, nshards: int) -> tuple[int, int]:
    """Equal-count plan for collectives that need equal counts (ncclScatter /
    ncclGather, rccl.h:745-769): returns (per_shard_bytes, padded_total)."""
    per = -(-nbytes // nshards)
    per = -(-per // BLOCK) * BLOCK
    return per, per * nshards


def ctr_add(counter: bytes, blocks: int, wrap64: bool = False) -> bytes:
    """128-bit big-endian counter + blocks (or 64-bit add on the low half,
    RFC 3686 / AES-NI layout of reference aesni.c:139-143)."""
    c = int.from_bytes(bytes(counter), "big")
    if wrap64:
        hi, lo = c >> 64, c & ((1 << 64) - 1)
        return ((hi << 64) | ((lo + blocks) & ((1 << 64) - 1))).to_bytes(16, "big")
    return ((c + blocks) % (1 << 128)).to_bytes(16, "big")


def rfc3686_block(nonce: bytes, ivec: bytes) -> bytes:
    return bytes(nonce) + bytes(ivec) + b"\x00\x00\x00\x01"


def chunks(nbytes: int, chunk: int) -> list[tuple[int, int]]:
    """Streaming plan: (offset, length) pieces of at most ``chunk`` bytes,
    16-aligned except the last."""
    chunk = max(BLOCK, chunk - chunk % BLOCK)
    return [(o, min(chunk, nbytes - o)) for o in range(0, nbytes, chunk)]


def cbc_halos(ciphertext: bytes, iv: bytes, shards: list[Shard]) -> list[bytes]:
    """Per shard: the IV to use for independent CBC decryption (the previous
    shard's last ciphertext block, or the stream IV for shard 0)."""
    return [bytes(iv) if s.offset == 0 else bytes(ciphertext[s.offset - BLOCK: s.offset]) for s in shards]
