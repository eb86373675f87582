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

IMPLS = {"auto": 0, "ttable": 1, "bitslice": 2, "split": 3}  # otc.h OTC_IMPL_*


def _impl(impl) -> int:
    if isinstance(impl, int):
        return impl
    try:
        return IMPLS[impl]
    except KeyError:
        raise ValueError(f"impl must be one of {list(IMPLS)}") from None


_IMPL_NAMES = {v: k for k, v in IMPLS.items()}


_PICK_MODES = {"ctr": 1, "ecb": 0, "dec": 2, "ecb-dec": 2, "cbc-dec": 2, "cfb-dec": 3, "seg-dec": 4, "seg-enc": 5}


def pick_impl(impl="auto", bits: int = 128, mode: str = "ctr", nbytes: int = 0) -> str:
    """The kernel family ``impl`` resolves to for a ``mode`` call ("ctr",
    "ecb" = ECB encryption, "dec" = ECB / CBC decryption, "cfb-dec") of ``nbytes`` with
    a ``bits``-bit key (the native routing rule)."""
    if mode not in _PICK_MODES:
        raise ValueError(f"mode must be one of {list(_PICK_MODES)}")
    r = _lib().otc_pick_impl(_impl(impl), int(bits), _PICK_MODES[mode], int(nbytes))
    if r < 0:
        raise ValueError(f"bad impl {impl!r}")
    return _IMPL_NAMES[r]


def last_impl() -> str:
    """What the calling thread's last ``ctr`` / ``ecb_*`` call actually ran."""
    return _IMPL_NAMES[_lib().otc_last_impl()]


def split_fallback_reason() -> str:
    """Why the calling thread's last split / bitsliced-claim request ran the
    T-table alone ("" if it did not fall back; otc.h otc_split_fallback_reason)."""
    return (_lib().otc_split_fallback_reason() or b"").decode()


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


def _run(x: torch.Tensor, out: torch.Tensor, call, inplace_ok: bool = True):
    """call(in_ptr, out_ptr) -> rc.  The kernels move 16 bytes per lane, so the
    native API requires 16-byte aligned buffers; a misaligned tensor (e.g. a
    byte slice ``t[3:]``) is staged through an aligned temporary (torch's
    allocator aligns every fresh allocation) and copied back.  Modes whose
    parallel kernel reads ciphertext block i-1 while block i-1's output is
    written (CBC / CFB decryption, ``inplace_ok=False``) run in place through
    a copy of the input."""
    xp, op = x.data_ptr(), out.data_ptr()
    if not inplace_ok and xp == op and _nbytes(x) > 16:
        x = _bytes(x).clone()
        xp = x.data_ptr()
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


BATCH_TILES = (256, 128, 64)  # tile sizes in blocks the batch kernel supports (otc.h)
BATCH_ALIGNED = 0x80000000  # otc.h OTC_BATCH_ALIGNED
BATCH_ALIGN_MIN_TILES = 6  # counter-aligned tiling pays once (n+1) x 133 < n x 160 lookups
# relative cost per tile block slot, measured on MI355X with 16384 x 4 KiB
# messages (960 / 946 / 910 GB/s at 256 / 128 / 64 blocks per tile,
# profiles/r1/batch_ctr_tiles.jsonl): fewer blocks per lane hide less LDS latency
BATCH_TILE_COST = {256: 1.0, 128: 1.015, 64: 1.055}


class CtrStream:
    """Resumable AES-CTR over device tensors with the PolarSSL context
    semantics (reference aes-modes/aes.c:869-900): the stream may be split at
    ANY byte across ``update`` calls and the result equals one-shot ``ctr``.
    The context (``nonce_counter``, ``stream_block``, ``nc_off``) is host
    state; ``state()`` / ``CtrStream.from_state`` checkpoint and resume it.

    Tensors may start at any byte (slices): the native call handles a head
    from ``stream_block``, a misaligned body with the funnel-shift kernel and a
    tail whose keystream block is kept for the next call."""

    def __init__(self, key: bytes, nonce_counter: bytes, impl="auto"):
        self._key = bytes(key)
        self._k = expand_key(self._key)
        self._impl = _impl(impl)
        self.ctx = _native.OtcCtrCtx()
        _native.check(_lib().otc_aes_ctr_ctx_init(ctypes.byref(self.ctx), _b16(nonce_counter, "nonce_counter")),
                      "otc_aes_ctr_ctx_init")

    @property
    def nonce_counter(self) -> bytes:
        return bytes(self.ctx.nonce_counter)

    @property
    def stream_block(self) -> bytes:
        return bytes(self.ctx.stream_block)

    @property
    def nc_off(self) -> int:
        return int(self.ctx.nc_off)

    def state(self) -> dict:
        return {"nonce_counter": self.nonce_counter, "stream_block": self.stream_block, "nc_off": self.nc_off}

    @classmethod
    def from_state(cls, key: bytes, state: dict, impl="auto") -> "CtrStream":
        s = cls(key, state["nonce_counter"], impl)
        ctypes.memmove(s.ctx.stream_block, bytes(state["stream_block"]), 16)
        s.ctx.nc_off = int(state["nc_off"])
        return s

    def update(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        _check_dev(x, "x")
        out = _out_like(x, out)
        n = _nbytes(x)
        if n == 0:
            return out
        xp, op = x.data_ptr(), out.data_ptr()
        target = out
        if xp % 16 != op % 16:  # the native call needs a common alignment: stage the output
            tmp = torch.empty(n + 16, dtype=torch.uint8, device=x.device)
            off = (xp - tmp.data_ptr()) % 16
            target = tmp[off:off + n]
        with torch.cuda.device(x.device):
            rc = _lib().otc_aes_ctr_stream(ctypes.byref(self.ctx), ctypes.byref(self._k), n, xp, target.data_ptr(),
                                           self._impl, _stream(x))
        _native.check(rc, "otc_aes_ctr_stream")
        if target is not out:
            _bytes(out).copy_(target)
        return out


def _pick_tile(nbytes) -> int:
    """Tile size minimising (tile slots issued) x (cost per slot)."""
    best, best_cost = 256, None
    for t in BATCH_TILES:
        slots = int(((nbytes + 16 * t - 1) // (16 * t)).sum()) * t
        cost = slots * BATCH_TILE_COST[t]
        if best_cost is None or cost < best_cost:
            best, best_cost = t, cost
    return best


class CtrBatch:
    """A planned batch of independent AES-CTR messages -- own buffers, key and
    counter each -- executed by ONE kernel launch per key size
    (``otc_aes_ctr_batch``).

    The serving shape: thousands of packets / sectors / objects of a few KiB.
    One ``ctr()`` launch per message is launch-bound (microseconds of host and
    dispatch work per message) and puts a few workgroups on a 256-CU chip; the
    batch kernel instead deals 4 KiB tiles of all messages to persistent
    workgroups, one per CU.  Planning (validation, descriptors, tile map, key
    schedules; one pinned H2D copy) happens once here; ``run()`` only launches,
    so it can be replayed with new data in the same buffers, and captured in a
    HIP graph.

    xs / outs: GPU tensors (contiguous, 16-byte aligned; ``outs[i] is xs[i]``
    for in place); keys: AES keys (16/24/32 bytes) selected per message by
    ``key_index`` (default: keys[i] for message i); counters: the 16-byte
    initial counter block of every message (128-bit big-endian increment);
    tile_blocks: 64 / 128 / 256 blocks per tile (default: picked from the
    message sizes).  Distinct messages must not overlap.
    """

    def __init__(self, xs, keys, counters, outs=None, key_index=None, tile_blocks=None):
        import numpy as np

        n = len(xs)
        if len(counters) != n:
            raise ValueError("one counter per message")
        if outs is None:
            outs = [torch.empty_like(x) for x in xs]
        if len(outs) != n:
            raise ValueError("one output per message")
        if key_index is None:
            if len(keys) != n:
                raise ValueError("one key per message, or pass key_index")
            key_index = range(n)
        kidx = np.fromiter((int(k) for k in key_index), dtype=np.int64, count=n)
        if n and (kidx.min() < 0 or kidx.max() >= len(keys)):
            raise ValueError("key_index out of range")
        self.outs = list(outs)
        self._keep = list(xs)  # descriptors hold raw addresses: keep the tensors alive
        self._launches = []
        self.device = xs[0].device if n else None
        self.ntiles, self.tile_blocks = 0, tile_blocks or 256
        if n == 0:
            return
        desc = np.zeros((n, 6), dtype=np.uint64)  # in, out, nbytes, ctr_hi, ctr_lo, key
        for i, (x, o) in enumerate(zip(xs, outs)):
            _check_dev(x, f"xs[{i}]")
            _check_dev(o, f"outs[{i}]")
            if x.device != self.device or o.device != self.device:
                raise ValueError("all messages must be on one device")
            nb = _nbytes(x)
            if _nbytes(o) != nb:
                raise ValueError(f"outs[{i}] must have the byte size of xs[{i}]")
            pi, po = x.data_ptr(), o.data_ptr()
            if nb and (pi % 16 or po % 16):
                raise ValueError(f"message {i}: batch buffers must be 16-byte aligned (clone a sliced tensor)")
            if pi != po and pi < po + nb and po < pi + nb:
                raise ValueError(f"message {i}: input and output overlap partially")
            c = bytes(counters[i])
            if len(c) != 16:
                raise ValueError(f"counters[{i}] must be 16 bytes")
            desc[i, :5] = (pi, po, nb, int.from_bytes(c[:8], "big"), int.from_bytes(c[8:], "big"))
        desc[:, 5] = kidx.astype(np.uint64)

        self._build(desc, keys, kidx, tile_blocks)

    @classmethod
    def packed(cls, buf: torch.Tensor, lengths, keys, counters, out: torch.Tensor | None = None, offsets=None,
               key_index=None, tile_blocks=None) -> "CtrBatch":
        """Messages packed in ONE device buffer (the usual serving layout):
        message i is ``buf[offsets[i] : offsets[i] + lengths[i]]`` (offsets
        default to back-to-back 16-byte aligned slots) and lands at the same
        offset of ``out`` (default: a new buffer; ``out is buf`` for in
        place).  counters: (n, 16) uint8 array / tensor or a list of 16-byte
        blocks.  Planning is vectorised (no per-message Python work); the
        outputs are ``self.out``."""
        import numpy as np

        nb = _nbytes(buf)
        lens = np.asarray(lengths, dtype=np.int64).reshape(-1)
        n = lens.size
        if offsets is None:
            offs = np.zeros(n, dtype=np.int64)
            if n > 1:
                offs[1:] = np.cumsum((lens[:-1] + 15) // 16 * 16)
        else:
            offs = np.asarray(offsets, dtype=np.int64).reshape(-1)
        if offs.size != n:
            raise ValueError("one offset per message")
        if n and ((lens < 0).any() or (offs < 0).any() or (offs + lens > nb).any()):
            raise ValueError("messages must lie inside the buffer")
        if n and (offs % 16).any():
            raise ValueError("message offsets must be multiples of 16")
        nz = np.nonzero(lens)[0]  # disjoint messages (empty ones occupy nothing)
        if nz.size > 1:
            so, sl = offs[nz], lens[nz]
            o = np.argsort(so, kind="stable")
            if ((so[o][:-1] + sl[o][:-1]) > so[o][1:]).any():
                raise ValueError("messages overlap")
        ctr = counters.cpu().numpy() if isinstance(counters, torch.Tensor) else counters
        if isinstance(ctr, np.ndarray):
            c = np.ascontiguousarray(ctr, dtype=np.uint8).reshape(-1, 16)
        else:
            if len(ctr) != n or any(len(bytes(x)) != 16 for x in ctr):
                raise ValueError("one 16-byte counter per message")
            c = np.frombuffer(b"".join(bytes(x) for x in ctr), dtype=np.uint8).reshape(-1, 16)
        if c.shape[0] != n:
            raise ValueError("one 16-byte counter per message")
        if key_index is None:
            if len(keys) != n:
                raise ValueError("one key per message, or pass key_index")
            kidx = np.arange(n, dtype=np.int64)
        else:
            kidx = np.asarray(key_index, dtype=np.int64).reshape(-1)
            if kidx.size != n:
                raise ValueError("one key index per message")
        if n and (kidx.min() < 0 or kidx.max() >= len(keys)):
            raise ValueError("key_index out of range")
        _check_dev(buf, "buf")
        out = _out_like(buf, out)
        pi, po = buf.data_ptr(), out.data_ptr()
        if (pi | po) % 16:
            raise ValueError("buf / out must be 16-byte aligned")
        if pi != po and pi < po + nb and po < pi + nb:
            raise ValueError("buf and out overlap partially")
        self = cls.__new__(cls)
        self.out = out
        self.outs = [out]
        self._keep = [buf]
        self._launches = []
        self.device = buf.device
        if n == 0:
            self.ntiles, self.tile_blocks = 0, tile_blocks or 256
            return self
        desc = np.zeros((n, 6), dtype=np.uint64)
        desc[:, 0] = np.uint64(pi) + offs.astype(np.uint64)
        desc[:, 1] = np.uint64(po) + offs.astype(np.uint64)
        desc[:, 2] = lens.astype(np.uint64)
        desc[:, 3] = c[:, :8].copy().view(">u8").reshape(-1).astype(np.uint64)
        desc[:, 4] = c[:, 8:].copy().view(">u8").reshape(-1).astype(np.uint64)
        desc[:, 5] = kidx.astype(np.uint64)
        self._build(desc, keys, kidx, tile_blocks)
        return self

    def _build(self, desc, keys, kidx, tile_blocks):
        """Tile map + key schedules + descriptors -> one pinned upload."""
        import numpy as np

        if tile_blocks is None:
            tile_blocks = _pick_tile(desc[:, 2])
        if tile_blocks not in BATCH_TILES:
            raise ValueError(f"tile_blocks must be one of {BATCH_TILES}")
        self.tile_blocks = tile_blocks
        tile_bytes = 16 * tile_blocks
        # messages of many tiles use counter-aligned tiles (otc.h
        # OTC_BATCH_ALIGNED): one partial tile more, but rounds 1-2 are mostly
        # computed once per tile (133 instead of 160 lookups per block)
        tb = np.uint64(tile_blocks)
        aligned = (desc[:, 2] + np.uint64(15)) // np.uint64(16) >= np.uint64(BATCH_ALIGN_MIN_TILES) * tb
        shift = np.where(aligned, desc[:, 4] % tb, np.uint64(0)).astype(np.uint64)
        align = np.where(aligned, np.uint64(BATCH_ALIGNED) | shift, np.uint64(0)).astype(np.uint64)
        desc[:, 5] = (desc[:, 5] & np.uint64(0xFFFFFFFF)) | (align << np.uint64(32))
        self.aligned_msgs = int(aligned.sum())
        ek = [expand_key(k) for k in keys]
        key_blob = b"".join(bytes(k) for k in ek)  # otc_aes_key[] (256 B each)
        nr_msg = np.array([k.nr for k in ek], dtype=np.int64)[kidx]
        parts, launches, off = [key_blob], [], len(key_blob)

        def add(b: bytes) -> int:
            nonlocal off
            pad = (-off) % 16
            if pad:
                parts.append(bytes(pad))
                off += pad
            at = off
            parts.append(b)
            off += len(b)
            return at

        for nr in (10, 12, 14):
            sel = np.nonzero(nr_msg == nr)[0]
            if not len(sel):
                continue
            d = desc[sel]
            sh = (d[:, 5] >> np.uint64(32)) & np.uint64(0xFFFF)
            tiles = np.where(d[:, 2] > 0, (d[:, 2] + np.uint64(16) * sh + np.uint64(tile_bytes - 1)) // np.uint64(tile_bytes),
                             np.uint64(0))
            ntiles = int(tiles.sum())
            if ntiles == 0:
                continue
            first = np.zeros(len(sel), dtype=np.uint64)
            first[1:] = np.cumsum(tiles)[:-1]
            tmap = np.repeat(np.arange(len(sel), dtype=np.uint32), tiles.astype(np.int64))
            assert tmap.size == ntiles and int(tmap.max()) < len(sel)
            launches.append((add(d.tobytes()), add(first.tobytes()), add(tmap.tobytes()), ntiles, nr))
        host = torch.frombuffer(bytearray(b"".join(parts)), dtype=torch.uint8).pin_memory()
        self._plan = host.to(self.device, non_blocking=True)
        self._ready = torch.cuda.Event()
        self._ready.record(torch.cuda.current_stream(self.device))
        self._launches = launches
        self.ntiles = sum(t for *_, t, _ in launches)

    def run(self, stream=None):
        """Launch the batch on ``stream`` (default: the current stream);
        returns the list of outputs."""
        if not self._launches:
            return self.outs
        st = stream or torch.cuda.current_stream(self.device)
        st.wait_event(self._ready)
        base = self._plan.data_ptr()
        lib = _lib()
        with torch.cuda.device(self.device):
            for o_desc, o_first, o_map, ntiles, nr in self._launches:
                rc = lib.otc_aes_ctr_batch(base + o_desc, base, base + o_map, base + o_first, ntiles,
                                           self.tile_blocks, nr, ctypes.c_void_p(st.cuda_stream))
                _native.check(rc, "otc_aes_ctr_batch")
        return self.outs


def ctr_batch(xs, keys, counters, outs=None, key_index=None, tile_blocks=None):
    """Plan and run a ``CtrBatch`` once."""
    return CtrBatch(xs, keys, counters, outs=outs, key_index=key_index, tile_blocks=tile_blocks).run()


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


def ecb_decrypt(x: torch.Tensor, key: bytes, out=None, impl="auto") -> torch.Tensor:
    """ECB decryption: the T-table inverse cipher, the bitsliced one (the
    forward S-box as S^-1 = L S L), or both concurrently ("split").  "auto":
    the split from 2 GiB, the persistent T-table claim kernel alone from 512
    MiB, the grid T-table below (engine.cpp pick_ecb_impl / split_form)."""
    _check_dev(x, "x")
    out = _out_like(x, out)
    k = expand_key(key, decrypt=True)
    with torch.cuda.device(x.device):
        rc = _run(x, out, lambda ip, op: _lib().otc_aes_ecb(ip, op, _nbytes(x), ctypes.byref(k), _impl(impl),
                                                           _stream(x)))
    _native.check(rc, "otc_aes_ecb(decrypt)")
    return out


def cbc_decrypt(x: torch.Tensor, key: bytes, iv: bytes, out=None, impl="auto") -> torch.Tensor:
    """Parallel CBC decryption (kernel choice as ecb_decrypt).  In place
    (out=x) runs through a copy of the input: block i needs ciphertext block
    i-1, which its own output overwrites."""
    _check_dev(x, "x")
    out = _out_like(x, out)
    k = expand_key(key, decrypt=True)
    with torch.cuda.device(x.device):
        rc = _run(x, out, lambda ip, op: _lib().otc_aes_cbc_decrypt_impl(ip, op, _nbytes(x), ctypes.byref(k),
            _b16(iv, "iv"), _impl(impl), _stream(x)), inplace_ok=False)
    _native.check(rc, "otc_aes_cbc_decrypt")
    return out


def cbc_encrypt_segments(x: torch.Tensor, key: bytes, iv0: bytes, segment_bytes: int, out=None,
                         impl="auto") -> torch.Tensor:
    """CBC encryption of independent contiguous segments; segment s uses
    IV = iv0 + s (128-bit BE), one serial chain per segment, one chain per
    lane on the T-table kernels for every ``impl`` (the persistent claim
    kernel from 1 GiB, the grid kernel
    below; a VALU kernel for this mode lost at every size and was removed).  A
    single segment is exact serial CBC on ONE lane -- use
    ``models.AES.cbc_encrypt`` (routes exact single-stream encryption to the
    host AES-NI chain) unless the buffer is small.  May run in place."""
    return _seg_call("otc_aes_cbc_encrypt_segments_impl", x, key, iv0, segment_bytes, out, True, impl)


def cbc_decrypt_segments(x: torch.Tensor, key: bytes, iv0: bytes, segment_bytes: int, out=None,
                         impl="auto") -> torch.Tensor:
    """Inverse of ``cbc_encrypt_segments``: fully parallel.  ``impl``:
    "ttable", "bitslice" (the bitsliced claim kernel alone), "split" (both at
    once), "auto" = split from 2 GiB of power-of-two segments, the persistent
    T-table claim kernel from 512 MiB (other segment sizes: the T-table)."""
    _check_dev(x, "x")
    out = _out_like(x, out)
    n = _nbytes(x)
    if segment_bytes <= 0 or n % segment_bytes:
        raise ValueError("byte size must be a multiple of segment_bytes")
    k = expand_key(key, decrypt=True)
    with torch.cuda.device(x.device):
        rc = _run(x, out, lambda ip, op: _lib().otc_aes_cbc_decrypt_segments_impl(ip, op, segment_bytes,
            n // segment_bytes, ctypes.byref(k), _b16(iv0, "iv0"), _impl(impl), _stream(x)), inplace_ok=False)
    _native.check(rc, "otc_aes_cbc_decrypt_segments")
    return out


def cfb128_decrypt(x: torch.Tensor, key: bytes, iv: bytes, out=None, impl="auto") -> torch.Tensor:
    """Parallel CFB128 decryption, P_i = C_i ^ E(C_{i-1}) (encryption key).
    ``impl``: "ttable", "bitslice" (the forward bitsliced cipher on the input
    shifted one block), "split" (both at once, as ECB encryption) or "auto"
    (as ecb_decrypt).  In place runs through a copy of the input."""
    _check_dev(x, "x")
    out = _out_like(x, out)
    k = expand_key(key)
    with torch.cuda.device(x.device):
        rc = _run(x, out, lambda ip, op: _lib().otc_aes_cfb128_decrypt_impl(ip, op, _nbytes(x), ctypes.byref(k),
            _b16(iv, "iv"), _impl(impl), _stream(x)), inplace_ok=False)
    _native.check(rc, "otc_aes_cfb128_decrypt")
    return out


def _seg_call(fn_name: str, x: torch.Tensor, key: bytes, iv0: bytes, segment_bytes: int, out, inplace_ok: bool,
              impl="auto"):
    _check_dev(x, "x")
    out = _out_like(x, out)
    n = _nbytes(x)
    if segment_bytes <= 0 or segment_bytes % 16 or n % segment_bytes:
        raise ValueError("segment_bytes must be a positive multiple of 16 dividing the byte size")
    k = expand_key(key)
    with torch.cuda.device(x.device):
        rc = _run(x, out, lambda ip, op: getattr(_lib(), fn_name)(ip, op, segment_bytes, n // segment_bytes,
                  ctypes.byref(k), _b16(iv0, "iv0"), _impl(impl), _stream(x)), inplace_ok=inplace_ok)
    _native.check(rc, fn_name)
    return out


def cfb128_encrypt_segments(x: torch.Tensor, key: bytes, iv0: bytes, segment_bytes: int, out=None,
                            impl="auto") -> torch.Tensor:
    """CFB128 encryption of independent segments (IV_s = iv0 + s), one
    serial chain per segment (``impl`` as ``cbc_encrypt_segments``)."""
    return _seg_call("otc_aes_cfb128_encrypt_segments_impl", x, key, iv0, segment_bytes, out, True, impl)


def cfb128_decrypt_segments(x: torch.Tensor, key: bytes, iv0: bytes, segment_bytes: int, out=None,
                            impl="auto") -> torch.Tensor:
    """Inverse of ``cfb128_encrypt_segments``: fully parallel (``impl`` as
    ``cbc_decrypt_segments``)."""
    _check_dev(x, "x")
    out = _out_like(x, out)
    n = _nbytes(x)
    if segment_bytes <= 0 or segment_bytes % 16 or n % segment_bytes:
        raise ValueError("segment_bytes must be a positive multiple of 16 dividing the byte size")
    k = expand_key(key)
    with torch.cuda.device(x.device):
        rc = _run(x, out, lambda ip, op: _lib().otc_aes_cfb128_decrypt_segments_impl(ip, op, segment_bytes,
            n // segment_bytes, ctypes.byref(k), _b16(iv0, "iv0"), _impl(impl), _stream(x)), inplace_ok=False)
    _native.check(rc, "otc_aes_cfb128_decrypt_segments")
    return out
