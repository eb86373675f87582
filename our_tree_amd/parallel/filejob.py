"""Resumable file-to-file streaming (checkpoint/resume:
"for 1 TiB streamed jobs, a resume cursor (chunk index, counter) so an
interrupted run restarts at a chunk boundary").

The reference keeps only in-memory cipher-stream state (arc4_context x/y/m,
CBC iv, CFB iv_off, CTR nc_off/stream_block -- /root/reference/arc4.c:93-94,
aes.c:792-897) and has no on-disk checkpoint.  Here a job over a file of any
size (bigger than host RAM and HBM) is processed chunk by chunk through the
pinned GPU pipeline (``StreamEngine``, csrc/hip/engine.cpp); after every chunk
the output range is flushed and a small JSON cursor is replaced atomically
(write + fsync + rename).  Restarting the same job resumes at the first chunk
not yet recorded; each chunk is self-contained because the mode state at a
chunk boundary is derivable from the inputs alone:

* CTR: counter = ctr0 + offset/16 (128-bit add) -- ``block_offset``;
* CBC decrypt: iv = the previous ciphertext block, read from the source;
* ECB: stateless.

The cursor stores a SHA-256 digest of (mode, key, iv) -- never the key -- and
the sizes, so a cursor from a different job is refused instead of silently
producing a mixed output.
"""
from __future__ import annotations

import hashlib
import json
import os
from typing import Callable, Optional

import numpy as np

CURSOR_VERSION = 1


def _digest(mode: str, key: bytes, iv: bytes) -> str:
    return hashlib.sha256(b"otc-filejob\0" + mode.encode() + b"\0" + bytes(key) + bytes(iv)).hexdigest()


def _write_cursor(path: str, cur: dict):
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(cur, f)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


def read_cursor(path: str) -> Optional[dict]:
    try:
        with open(path) as f:
            return json.load(f)
    except FileNotFoundError:
        return None


def gpu_backend(device: int = 0, chunk_bytes: int = 256 << 20, impl: str = "auto"):
    """Backend running every chunk through the native pinned pipeline."""
    from .stream import StreamEngine

    eng = StreamEngine(device=device, chunk_bytes=min(chunk_bytes, 256 << 20))

    def run(mode, src, dst, key, iv, block_offset):
        eng.run(mode, src, dst, key, iv, block_offset=block_offset, impl=impl)

    run.close = eng.close
    return run


def cpu_backend():
    """Backend on the C oracle (tests; no GPU needed)."""
    from ..models import cpu_ref

    def run(mode, src, dst, key, iv, block_offset):
        data = src.tobytes()
        if mode == "ctr":
            out = cpu_ref.ctr(key, iv, data, block_offset)
        elif mode == "ecb":
            out = cpu_ref.ecb(key, data)
        elif mode == "cbc-dec":
            out = cpu_ref.cbc(key, iv, data, decrypt=True)
        else:
            raise ValueError(mode)
        dst[:] = np.frombuffer(out, dtype=np.uint8)

    return run


def crypt_file(src_path: str, dst_path: str, key: bytes, iv_or_counter: bytes = bytes(16), mode: str = "ctr",
               chunk_bytes: int = 1 << 30, cursor_path: Optional[str] = None,
               backend: Optional[Callable] = None, max_chunks: Optional[int] = None) -> dict:
    """Encrypt/decrypt ``src_path`` into ``dst_path`` chunk by chunk, resumably.

    mode: "ctr" (any length), "ecb" / "cbc-dec" (length % 16 == 0).
    cursor_path: defaults to ``dst_path + ".cursor"``; removed on completion.
    max_chunks: process at most this many chunks in this call (simulates an
    interruption; the cursor then points at the next chunk).
    Returns {"done": bool, "next_chunk", "chunks", "bytes_done", "resumed_from"}.
    """
    if mode not in ("ctr", "ecb", "cbc-dec"):
        raise ValueError("mode must be ctr, ecb or cbc-dec")
    if chunk_bytes <= 0 or chunk_bytes % 16:
        raise ValueError("chunk_bytes must be a positive multiple of 16")
    iv_or_counter = bytes(iv_or_counter)
    if len(iv_or_counter) != 16:
        raise ValueError("iv/counter must be 16 bytes")
    n = os.path.getsize(src_path)
    if mode != "ctr" and n % 16:
        raise ValueError(f"{mode} needs a multiple of 16 bytes")
    cursor_path = cursor_path or dst_path + ".cursor"
    nchunks = (n + chunk_bytes - 1) // chunk_bytes
    ident = {"version": CURSOR_VERSION, "mode": mode, "size": n, "chunk_bytes": chunk_bytes,
             "digest": _digest(mode, key, iv_or_counter)}

    start = 0
    cur = read_cursor(cursor_path)
    if cur is not None:
        if any(cur.get(k) != v for k, v in ident.items()):
            raise ValueError(f"cursor {cursor_path} belongs to a different job; remove it to restart")
        start = int(cur["next_chunk"])
        if not os.path.exists(dst_path) or os.path.getsize(dst_path) != n:
            raise ValueError("cursor present but the output file is missing or has the wrong size")
    else:
        with open(dst_path, "wb") as f:  # fresh job: size the output (sparse)
            f.truncate(n)
        _write_cursor(cursor_path, {**ident, "next_chunk": 0, "bytes_done": 0})

    own_backend = backend is None
    if own_backend:
        backend = gpu_backend(chunk_bytes=chunk_bytes)
    try:
        if n == 0:
            os.remove(cursor_path)
            return {"done": True, "next_chunk": 0, "chunks": 0, "bytes_done": 0, "resumed_from": start}
        src = np.memmap(src_path, dtype=np.uint8, mode="r", shape=(n,))
        dst = np.memmap(dst_path, dtype=np.uint8, mode="r+", shape=(n,))
        stop = nchunks if max_chunks is None else min(nchunks, start + max_chunks)
        for c in range(start, stop):
            off = c * chunk_bytes
            end = min(n, off + chunk_bytes)
            iv, bo = iv_or_counter, 0
            if mode == "ctr":
                bo = off // 16
            elif mode == "cbc-dec" and off > 0:
                iv = bytes(src[off - 16:off])
            # contiguous copies: the engine pins/stages host memory itself
            sin = np.ascontiguousarray(src[off:end])
            sout = np.empty_like(sin)
            backend(mode, sin, sout, key, iv, bo)
            dst[off:end] = sout
            dst.flush()
            _write_cursor(cursor_path, {**ident, "next_chunk": c + 1, "bytes_done": end})
        del src, dst
        done = stop == nchunks
        if done:
            os.remove(cursor_path)
        return {"done": done, "next_chunk": stop, "chunks": nchunks,
                "bytes_done": min(n, stop * chunk_bytes), "resumed_from": start}
    finally:
        if own_backend and hasattr(backend, "close"):
            backend.close()
