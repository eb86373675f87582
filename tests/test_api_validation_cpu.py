"""Fault injection against the native device API (csrc/hip/engine.cpp, C API
csrc/include/otc.h) without a GPU: every bad argument -- misaligned or null
pointers, partial overlaps, bad lengths, wrong key schedules, size overflow --
must be rejected with OTC_ERR_ARG and a message *before* any HIP call, so the
fake pointers below are never dereferenced.  (The reference checks nothing:
AES.cu:217-254 ignores every CUDA return code; SURVEY.md section 5 "Failure
detection".)"""
import ctypes

import pytest

from our_tree_amd import _native

ERR_ARG = -1
ENC, DEC = 1, 0
A = 0x7F0000000000  # fake, 16-byte aligned device addresses (never touched)


@pytest.fixture(scope="module")
def lib():
    if not _native.gpu_lib_available():
        pytest.skip("libotc.so not built")
    return _native.require_gpu_lib()


def key(lib, bits=128, d=ENC):
    k = _native.OtcAesKey()
    assert lib.otc_aes_key_init(ctypes.byref(k), _native.as_u8p(bytes(range(bits // 8))), bits, d) == 0
    return k


def err(lib) -> str:
    return lib.otc_last_error().decode()


def c16():
    return (ctypes.c_uint8 * 16)()


def test_key_init_rejects_bad_sizes(lib):
    k = _native.OtcAesKey()
    assert lib.otc_aes_key_init(ctypes.byref(k), _native.as_u8p(bytes(20)), 160, ENC) == ERR_ARG
    assert "128/192/256" in err(lib)


@pytest.mark.parametrize("inp,out,what", [
    (A + 1, A + 4096, "aligned"),
    (A, A + 4096 + 8, "aligned"),
    (None, A, "null"),
    (A, None, "null"),
    (A, A + 16, "overlap"),
    (A + 32, A, "overlap"),
])
def test_ctr_rejects_bad_buffers(lib, inp, out, what):
    k = key(lib)
    rc = lib.otc_aes_ctr(inp, out, 1024, ctypes.byref(k), c16(), 0, 0, None)
    assert rc == ERR_ARG and what in err(lib)


def test_zero_length_is_a_noop(lib):
    k = key(lib)
    assert lib.otc_aes_ctr(None, None, 0, ctypes.byref(k), c16(), 0, 0, None) == 0
    assert lib.otc_aes_ecb(A + 3, A + 5, 0, ctypes.byref(k), 0, None) == 0


def test_ecb_length_and_alignment(lib):
    k = key(lib)
    assert lib.otc_aes_ecb(A, A + 4096, 17, ctypes.byref(k), 0, None) == ERR_ARG
    assert "multiple of 16" in err(lib)
    assert lib.otc_aes_ecb(A + 8, A + 4096, 32, ctypes.byref(k), 0, None) == ERR_ARG


def test_wrong_schedule_direction(lib):
    kd = key(lib, 256, DEC)
    assert lib.otc_aes_ctr(A, A + 4096, 64, ctypes.byref(kd), c16(), 0, 0, None) == ERR_ARG
    assert "encryption schedule" in err(lib)
    ke = key(lib, 192, ENC)
    assert lib.otc_aes_cbc_decrypt(A, A + 4096, 64, ctypes.byref(ke), c16(), None) == ERR_ARG
    assert "decryption schedule" in err(lib)


def test_cbc_cfb_in_place_rules(lib):
    kd, ke = key(lib, 128, DEC), key(lib, 128, ENC)
    assert lib.otc_aes_cbc_decrypt(A, A, 64, ctypes.byref(kd), c16(), None) == ERR_ARG
    assert "in-place" in err(lib)
    assert lib.otc_aes_cfb128_decrypt(A, A, 64, ctypes.byref(ke), c16(), None) == ERR_ARG
    assert lib.otc_aes_cbc_decrypt_segments(A, A, 64, 4, ctypes.byref(kd), c16(), None) == ERR_ARG
    assert lib.otc_aes_cbc_decrypt(A, A + 4096, 64, ctypes.byref(kd), None, None) == ERR_ARG
    assert "null iv" in err(lib)


def test_segment_size_overflow(lib):
    k = key(lib)
    big = 1 << 62
    assert lib.otc_aes_cbc_encrypt_segments(A, A + 4096, big, 16, ctypes.byref(k), c16(), None) == ERR_ARG
    assert "overflow" in err(lib)
    assert lib.otc_aes_cbc_encrypt_segments(A, A + 4096, 20, 2, ctypes.byref(k), c16(), None) == ERR_ARG


def test_stream_ops_validation(lib):
    assert lib.otc_xor(A + 4, A + 4096, A + 8192, 64, None) == ERR_ARG
    assert lib.otc_xor(A, A + 4096, A + 4096 + 16, 64, None) == ERR_ARG  # b overlaps out
    assert lib.otc_checksum(A + 4, 64, A + 4096, None) == ERR_ARG
    assert lib.otc_checksum(A, 63, A + 4096, None) == ERR_ARG
    assert lib.otc_rc4_multi(A, 0, 4, 16, 0, None, A + 4096, None) == ERR_ARG
    assert lib.otc_rc4_multi(A, 257, 4, 16, 0, None, A + 4096, None) == ERR_ARG
    assert lib.otc_rc4_multi(A, 16, 4, 64, 0, A, A + 16, None) == ERR_ARG
    assert "overlap" in err(lib)
    assert lib.otc_fill_random(A + 2, 64, 1, None) == ERR_ARG


def test_engine_and_multi_reject_bad_arguments(lib):
    assert lib.otc_engine_run(None, 1, None, None, 16, None, None, 0, 0, None) == ERR_ARG
    st = _native.MultiStats() if hasattr(_native, "MultiStats") else None
    rc = lib.otc_multi_run(0, 0, 1, None, None, 16, None, None, 0, 0,
                           ctypes.byref(st) if st is not None else None)
    assert rc == ERR_ARG


@pytest.mark.parametrize("bits", [128, 192, 256])
@pytest.mark.parametrize("dec", [False, True])
def test_aesni_schedule_bytes_equal_kernel_schedule(lib, bits, dec):
    """otc_aesni.h passes AES-NI schedules straight to the kernels: the
    AES_*_Key_Expansion / AES_Key_Expansion_Dec bytes must equal the PolarSSL
    word schedule (otc_aes_key.rk) byte for byte."""
    from our_tree_amd.models import cpu_ref
    if not cpu_ref.aesni_supported():
        pytest.skip("no AES-NI on this CPU")
    kb = bytes((7 * i + 3) & 0xFF for i in range(bits // 8))
    sched, nr = cpu_ref.aesni_schedule(kb, decrypt=dec)
    k = _native.OtcAesKey()
    assert lib.otc_aes_key_init(ctypes.byref(k), _native.as_u8p(kb), bits, DEC if dec else ENC) == 0
    assert k.nr == nr
    assert bytes(k)[: 16 * (nr + 1)] == sched


def test_aesni_shaped_api_rejects_bad_rounds(lib):
    sched = (ctypes.c_uint8 * 240)()
    assert lib.otc_AES_ECB_encrypt(A, A + 4096, 64, sched, 11, None) == ERR_ARG
    assert "number_of_rounds" in err(lib)
    assert lib.otc_AES_CTR_encrypt(A + 1, A + 4096, c16(), c16(), 64, sched, 10, None) == ERR_ARG


class CtrMsg(ctypes.Structure):
    """Mirror of otc_ctr_msg (otc.h)."""
    _fields_ = [("inp", ctypes.c_uint64), ("out", ctypes.c_uint64), ("nbytes", ctypes.c_uint64),
                ("ctr_hi", ctypes.c_uint64), ("ctr_lo", ctypes.c_uint64), ("key", ctypes.c_uint32),
                ("align", ctypes.c_uint32)]


def test_ctr_batch_planner_and_python_plan_agree(lib):
    """The C host planner (otc_ctr_batch_plan) builds the tile map ops.CtrBatch
    builds with numpy: 4 KiB tiles, empty messages own none."""
    import numpy as np

    from our_tree_amd.ops import aes_ops

    sizes = [0, 1, 4096, 4097, 16, 0, 3 * 4096 + 15, 100000, 1504]
    msgs = (CtrMsg * len(sizes))(*[CtrMsg(0, 0, n, 0, 0, 0, 0) for n in sizes])
    fn = lib.otc_ctr_batch_plan
    fn.restype = ctypes.c_uint64
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    for tb in (64, 128, 256):
        nt = fn(msgs, len(sizes), tb, None, None)
        tmap = np.zeros(nt, np.uint32)
        first = np.zeros(len(sizes), np.uint64)
        assert fn(msgs, len(sizes), tb, tmap.ctypes.data, first.ctypes.data) == nt
        tiles = (np.array(sizes, np.uint64) + 16 * tb - 1) // (16 * tb)
        assert nt == tiles.sum()
        assert (tmap == np.repeat(np.arange(len(sizes), dtype=np.uint32), tiles.astype(np.int64))).all()
        assert first[0] == 0 and (first[1:] == np.cumsum(tiles)[:-1]).all()
    assert fn(msgs, len(sizes), 100, None, None) == 0
    # counter-aligned messages (OTC_BATCH_ALIGNED | shift) own ceil((bytes + 16 shift) / tile) tiles
    al = (CtrMsg * 2)(CtrMsg(0, 0, 4096 * 10, 0, 0, 0, 0x80000000 | 5), CtrMsg(0, 0, 4096 * 10, 0, 0, 0, 0x80000000))
    assert fn(al, 2, 256, None, None) == 11 + 10
    # tile choice: 4 KiB messages fill 256-block tiles exactly, 1 KiB ones 64-block tiles
    assert aes_ops._pick_tile(np.full(100, 4096, np.uint64)) == 256
    assert aes_ops._pick_tile(np.full(100, 1024, np.uint64)) == 64


def test_ctr_batch_rejects_bad_launch_args(lib):
    f = lib.otc_aes_ctr_batch
    assert f(A, A, A, A, 0, 256, 10, None) == 0  # nothing to do
    assert f(None, A, A, A, 4, 256, 10, None) == ERR_ARG and "null" in err(lib)
    assert f(A, A, A, A, 4, 256, 11, None) == ERR_ARG and "nr" in err(lib)
    assert f(A, A, A, A, 4, 100, 10, None) == ERR_ARG and "tile_blocks" in err(lib)
    assert f(A + 4, A, A, A, 4, 64, 10, None) == ERR_ARG and "misaligned" in err(lib)


def test_ctr_batch_python_validation_without_gpu():
    import torch

    from our_tree_amd import ops

    x = torch.zeros(16, dtype=torch.uint8)
    with pytest.raises(ValueError, match="one counter"):
        ops.CtrBatch([x], [bytes(16)], [])
    with pytest.raises(ValueError, match="GPU tensor"):
        ops.CtrBatch([x], [bytes(16)], [bytes(16)])
    with pytest.raises(ValueError, match="key_index"):
        ops.CtrBatch([x], [bytes(16)], [bytes(16)], key_index=[3])


def test_packed_batch_validation_without_gpu():
    """Packed-buffer planning rejects bad layouts before touching a device."""
    import torch

    from our_tree_amd import ops

    buf = torch.zeros(4096, dtype=torch.uint8)
    k, c = [bytes(16)], [bytes(16)] * 2
    with pytest.raises(ValueError, match="inside the buffer"):
        ops.CtrBatch.packed(buf, [4000, 200], k, c, key_index=[0, 0])
    with pytest.raises(ValueError, match="multiples of 16"):
        ops.CtrBatch.packed(buf, [10, 10], k, c, offsets=[0, 24], key_index=[0, 0])
    with pytest.raises(ValueError, match="overlap"):
        ops.CtrBatch.packed(buf, [100, 100], k, c, offsets=[0, 64], key_index=[0, 0])
    with pytest.raises(ValueError, match="16-byte counter"):
        ops.CtrBatch.packed(buf, [100, 100], k, [bytes(16)], key_index=[0, 0])
    with pytest.raises(ValueError, match="key_index"):
        ops.CtrBatch.packed(buf, [100, 100], k, c, key_index=[0, 1])
    with pytest.raises(ValueError, match="GPU tensor"):  # layout valid: only the device is wrong
        ops.CtrBatch.packed(buf, [100, 100], k, c, key_index=[0, 0])


def test_rccl_strategy_warns_on_pageable_host_buffers():
    """otc_multi_run strategy 1 enqueues every host copy from one thread, so
    pageable buffers serialise it: the Python API warns before the call
    (VERDICT r2 weak #8); the native call warns once on stderr too."""
    import numpy as np

    from our_tree_amd.parallel import stream as pstream

    x = np.zeros(4096, np.uint8)
    y = np.zeros(4096, np.uint8)
    assert pstream.pageable_buffers(x, y) == [0, 1]
    with pytest.warns(RuntimeWarning, match="host_in and host_out are pageable"):
        with pytest.raises(RuntimeError):  # no GPU here: the native call then refuses
            pstream.multi_gpu_run("ctr", x, y, bytes(16), bytes(16), ngpus=1, strategy="rccl")
