"""Numerics of every gfx950 kernel against the C oracle (csrc/cpu/aes.c, the
reference-compatible PolarSSL-API implementation) on random data, random keys,
odd lengths, unaligned counters and counter carries."""
import os

import pytest
import torch

from our_tree_amd import ops
from our_tree_amd.models import cpu_ref
from our_tree_amd.parallel import shard as sh

pytestmark = pytest.mark.gpu

IMPLS = ["ttable", "bitslice"]
KEYBITS = [128, 192, 256]


def rnd(n, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 256, (n,), dtype=torch.uint8, generator=g).to(dev)


def host(t):
    return t.cpu().numpy().tobytes()


@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("bits", KEYBITS)
@pytest.mark.parametrize("n", [16, 1000, 4096 * 16 + 5, (1 << 20) + 3, 3 * (1 << 20) + 16 * 777])
def test_ctr_matches_oracle(gpu, impl, bits, n):
    key = os.urandom(bits // 8)
    ctr0 = os.urandom(16)
    x = rnd(n, gpu, n + bits)
    y = ops.ctr(x, key, ctr0, impl=impl)
    torch.cuda.synchronize()
    assert host(y) == cpu_ref.ctr(key, ctr0, host(x))


@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("ctr_low", [0, 1, 2047, 2048, 0xFFFFFFFF, (1 << 64) - 5, (1 << 64) - 3000])
def test_ctr_counter_carries(gpu, impl, ctr_low):
    """Counters near 2^11 task boundaries, 2^32 and the 2^64 carry into the
    high half (128-bit add)."""
    key = os.urandom(16)
    hi = os.urandom(8)
    ctr0 = hi + ctr_low.to_bytes(8, "big")
    x = rnd(16 * 5000 + 9, gpu, 7)
    y = ops.ctr(x, key, ctr0, impl=impl)
    torch.cuda.synchronize()
    assert host(y) == cpu_ref.ctr(key, ctr0, host(x))


@pytest.mark.parametrize("bits", KEYBITS)
@pytest.mark.parametrize("ctr_low", [(1 << 64) - 70000, (1 << 16) - 2048 * 3 - 5, 0xFFFF0000 + 2048 * 17])
def test_ctr_bitslice_group_boundaries(gpu, bits, ctr_low):
    """The bitsliced kernel's counter caching precomputes rounds 1-2 per group
    of 32 tasks (counter bits 16+): many groups, a group straddling the 2^64
    carry into the high half, and groups starting mid-way."""
    key = os.urandom(bits // 8)
    ctr0 = os.urandom(8) + ctr_low.to_bytes(8, "big")
    x = rnd(16 * 300000 + 5, gpu, 13)
    y = ops.ctr(x, key, ctr0, impl="bitslice")
    torch.cuda.synchronize()
    assert host(y) == cpu_ref.ctr(key, ctr0, host(x))


def test_ctr_bitslice_wrap64_many_groups(gpu):
    """64-bit counter wrap (RFC 3686 layout) across group boundaries."""
    if not cpu_ref.aesni_supported():
        pytest.skip("no AES-NI on this host")
    key, nonce, ivec = os.urandom(16), os.urandom(4), b"\xff" * 4 + b"\xff\xfe\x00\x00"
    x = rnd(16 * 200000 + 7, gpu, 17)
    y = ops.ctr_rfc3686(x, key, nonce, ivec, impl="bitslice")
    torch.cuda.synchronize()
    assert host(y) == cpu_ref.aesni_ctr(key, nonce, ivec, host(x))


@pytest.mark.parametrize("impl", IMPLS)
def test_ctr_block_offset_and_inplace(gpu, impl):
    key = os.urandom(16)
    ctr0 = os.urandom(16)
    x = rnd(1 << 18, gpu, 3)
    ref = cpu_ref.ctr(key, ctr0, host(x), block_offset=123457)
    ops.ctr(x, key, ctr0, out=x, block_offset=123457, impl=impl)
    torch.cuda.synchronize()
    assert host(x) == ref


@pytest.mark.parametrize("impl", IMPLS)
def test_ctr_rfc3686(gpu, impl):
    """AES-NI counter layout with 64-bit wrap, against the AES-NI CPU baseline."""
    if not cpu_ref.aesni_supported():
        pytest.skip("no AES-NI on this host")
    key, nonce, ivec = os.urandom(32), os.urandom(4), b"\xff" * 4 + b"\xff\xff\xff\xf0"
    x = rnd(16 * 300 + 3, gpu, 11)
    y = ops.ctr_rfc3686(x, key, nonce, ivec, impl=impl)
    torch.cuda.synchronize()
    assert host(y) == cpu_ref.aesni_ctr(key, nonce, ivec, host(x))


@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("bits", KEYBITS)
def test_ecb_roundtrip(gpu, impl, bits):
    key = os.urandom(bits // 8)
    x = rnd(16 * 100003, gpu, bits)
    y = ops.ecb_encrypt(x, key, impl=impl)
    torch.cuda.synchronize()
    assert host(y) == cpu_ref.ecb(key, host(x), threads=8)
    z = ops.ecb_decrypt(y, key)
    torch.cuda.synchronize()
    assert torch.equal(z, x)


def test_fips197_appendix_c(gpu):
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    exp = {16: "69c4e0d86a7b0430d8cdb78070b4c55a", 24: "dda97ca4864cdfe06eaf70a0ec0d7191",
           32: "8ea2b7ca516745bfeafc49904b496089"}
    for kl, ct in exp.items():
        x = torch.tensor(list(pt), dtype=torch.uint8, device=gpu)
        for impl in IMPLS:
            assert host(ops.ecb_encrypt(x, bytes(range(kl)), impl=impl)).hex() == ct
        assert host(ops.ecb_decrypt(torch.tensor(list(bytes.fromhex(ct)), dtype=torch.uint8, device=gpu),
                                    bytes(range(kl)))) == pt


@pytest.mark.parametrize("bits", KEYBITS)
def test_cbc_decrypt(gpu, bits):
    key, iv = os.urandom(bits // 8), os.urandom(16)
    pt = os.urandom(16 * 70001)
    ct = cpu_ref.cbc(key, iv, pt)
    x = torch.frombuffer(bytearray(ct), dtype=torch.uint8).to(gpu)
    y = ops.cbc_decrypt(x, key, iv)
    torch.cuda.synchronize()
    assert host(y) == pt


@pytest.mark.parametrize("seg", [16, 48, 512, 4096, 16 * 37])
def test_cbc_segments_roundtrip(gpu, seg):
    key, iv0 = os.urandom(32), (2**128 - 3).to_bytes(16, "big")  # IV carry across segments
    nseg = 1000
    pt = os.urandom(seg * nseg)
    x = torch.frombuffer(bytearray(pt), dtype=torch.uint8).to(gpu)
    y = ops.cbc_encrypt_segments(x, key, iv0, seg)
    torch.cuda.synchronize()
    assert host(y) == cpu_ref.cbc_segments(key, iv0, pt, seg)
    z = ops.cbc_decrypt_segments(y, key, iv0, seg)
    torch.cuda.synchronize()
    assert host(z) == pt


def test_cbc_single_segment_is_exact_cbc(gpu):
    key, iv = os.urandom(16), os.urandom(16)
    pt = os.urandom(16 * 333)
    x = torch.frombuffer(bytearray(pt), dtype=torch.uint8).to(gpu)
    y = ops.cbc_encrypt_segments(x, key, iv, len(pt))
    assert host(y) == cpu_ref.cbc(key, iv, pt)


@pytest.mark.parametrize("bits", [128, 192, 256])
@pytest.mark.parametrize("seg", [16, 48, 512, 4096, 16 * 37])
def test_cfb128_segments_roundtrip(gpu, bits, seg):
    """CFB128 sector kernel (one serial chain per lane) vs the oracle per
    segment, every key size and every sector-kernel path (seg_blocks < 4, the
    4/8-block burst loops and their remainders), IV carry across segments;
    the parallel segment decryption inverts it (power-of-two and general
    segment lengths)."""
    key, iv0 = os.urandom(bits // 8), (2**128 - 5).to_bytes(16, "big")
    nseg = 700
    pt = os.urandom(seg * nseg)
    x = torch.frombuffer(bytearray(pt), dtype=torch.uint8).to(gpu)
    y = ops.cfb128_encrypt_segments(x, key, iv0, seg)
    torch.cuda.synchronize()
    assert host(y) == cpu_ref.cfb128_segments(key, iv0, pt, seg)
    z = ops.cfb128_decrypt_segments(y, key, iv0, seg)
    torch.cuda.synchronize()
    assert host(z) == pt
    ops.cfb128_encrypt_segments(x, key, iv0, seg, out=x)  # in place (lane-private chains)
    assert torch.equal(x, y)


def test_serial_chains_route_to_host(gpu):
    """Exact single-stream CBC / CFB128 encryption of a GPU tensor runs the
    host AES-NI chain (not one GPU lane) and equals the oracle; device_serial
    opts in to the one-lane kernel."""
    from our_tree_amd.models import AES

    key, iv = os.urandom(16), os.urandom(16)
    pt = os.urandom(16 * 4099)
    x = torch.frombuffer(bytearray(pt), dtype=torch.uint8).to(gpu)
    aes = AES(key)
    for mode, ref in (("cbc", cpu_ref.cbc(key, iv, pt)), ("cfb128", cpu_ref.cfb128(key, iv, pt))):
        enc = aes.cbc_encrypt if mode == "cbc" else aes.cfb128_encrypt
        y = enc(x, iv)
        assert y.device == x.device and host(y) == ref
        assert host(enc(x, iv, device_serial=True)) == ref
    assert host(aes.cfb128_decrypt(aes.cfb128_encrypt(x, iv, segment_bytes=16 * 4099), iv, segment_bytes=16 * 4099)) == pt


def test_cfb128_decrypt(gpu):
    key, iv = os.urandom(24), os.urandom(16)
    pt = os.urandom(16 * 5001)
    ct = cpu_ref.cfb128(key, iv, pt)
    x = torch.frombuffer(bytearray(ct), dtype=torch.uint8).to(gpu)
    assert host(ops.cfb128_decrypt(x, key, iv)) == pt


def test_sp800_38a_ctr_vector(gpu):
    key = bytes.fromhex("2b7e151628aed2a6abf7158809cf4f3c")
    ctr0 = bytes.fromhex("f0f1f2f3f4f5f6f7f8f9fafbfcfdfeff")
    pt = bytes.fromhex("6bc1bee22e409f96e93d7e117393172aae2d8a571e03ac9c9eb76fac45af8e51"
                       "30c81c46a35ce411e5fbc1191a0a52eff69f2445df4f9b17ad2b417be66c3710")
    exp = ("874d6191b620e3261bef6864990db6ce9806f66b7970fdff8617187bb9fffdff"
           "5ae4df3edbd5d35e5b4f09020db03eab1e031dda2fbe03d1792170a0f3009cee")
    x = torch.tensor(list(pt), dtype=torch.uint8, device=gpu)
    for impl in IMPLS:
        assert host(ops.ctr(x, key, ctr0, impl=impl)).hex() == exp


def test_sharded_ctr_equals_single_stream(gpu):
    """Device shards with planner offsets == one stream (the DP invariant)."""
    key, ctr0 = os.urandom(16), os.urandom(16)
    n = 16 * 12345 + 11
    x = rnd(n, gpu, 5)
    ref = host(ops.ctr(x, key, ctr0))
    parts = []
    for s in sh.plan(n, 7):
        parts.append(host(ops.ctr(x[s.offset:s.end].contiguous(), key, ctr0, block_offset=s.block_offset)))
    assert b"".join(parts) == ref


def test_xor_and_arc4(gpu):
    key = os.urandom(16)
    n = (1 << 20) + 13
    ks = cpu_ref.arc4_keystream(key, n)
    x = rnd(n, gpu, 9)
    k = torch.frombuffer(bytearray(ks), dtype=torch.uint8).to(gpu)
    y = ops.xor(x, k)
    assert host(y) == cpu_ref.arc4_crypt(host(x), ks)


@pytest.mark.parametrize("keylen,length,drop", [(16, 4096, 0), (5, 1000, 3), (256, 37, 768), (16, 1, 0), (16, 2, 0),
                                                (7, 3, 0), (16, 18, 0), (1, 19, 1), (16, 35, 0), (3, 8197, 0),
                                                (32, 100, 0), (8, 64, 16), (2, 40, 32), (32, 33, 768),
                                                (1, 64, 0), (4, 100, 256), (16, 50, 4096)])
def test_rc4_multi(gpu, keylen, length, drop):
    """every stream vs the oracle: lengths around the 16-byte blocks and the
    two-iteration write delay of the pipelined PRGA; short keys make the
    j == i / j == j' coincidences the pipeline corrects for frequent"""
    ns = 200
    keys = rnd(ns * keylen, gpu, keylen).view(ns, keylen)
    ks = ops.rc4_multi(keys, length, drop=drop)
    torch.cuda.synchronize()
    kh = keys.cpu().numpy()
    for s in range(ns):
        assert host(ks[s]) == cpu_ref.arc4_keystream(bytes(kh[s]), length, drop=drop)
    x = rnd(ns * length, gpu, 1).view(ns, length)
    y = ops.rc4_multi(keys, length, x=x, drop=drop)
    assert torch.equal(y, x ^ ks)


def test_rc4_multi_capped_launch(gpu):
    """10 workgroups (640 streams) per CU: the launch that reserves extra LDS
    to cap residency at 6 per CU (two rounds); sampled streams vs the oracle,
    first, last and strided"""
    ns = torch.cuda.get_device_properties(0).multi_processor_count * 640
    length = 48
    keys = rnd(ns * 16, gpu, 11).view(ns, 16)
    ks = ops.rc4_multi(keys, length)
    torch.cuda.synchronize()
    kh = keys.cpu().numpy()
    kso = ks.cpu().numpy()
    for s in list(range(0, ns, 997)) + [ns - 1]:
        assert kso[s].tobytes() == cpu_ref.arc4_keystream(bytes(kh[s]), length), s


def test_fill_and_checksum(gpu):
    a = torch.empty(1 << 20, dtype=torch.uint8, device=gpu)
    b = torch.empty(1 << 20, dtype=torch.uint8, device=gpu)
    ops.fill_random_(a, 5)
    ops.fill_random_(b, 5)
    assert torch.equal(a, b)
    assert ops.checksum(a) == ops.checksum(b)
    b[12345] ^= 1
    assert ops.checksum(a) != ops.checksum(b)


def test_errors_are_loud(gpu):
    x = rnd(17, gpu)
    with pytest.raises(RuntimeError):
        ops.ecb_encrypt(x, os.urandom(16))  # not a multiple of 16
    with pytest.raises(ValueError):
        ops.ctr(x, os.urandom(15), os.urandom(16))
    y = rnd(64, gpu)
    with pytest.raises(RuntimeError):  # partial overlap of input and output
        ops.cbc_decrypt(y[:48], os.urandom(16), os.urandom(16), out=y[16:])
    # exact in place is staged through a copy of the input (the kernel itself
    # would overwrite ciphertext block i-1 before block i reads it)
    key, iv = os.urandom(16), os.urandom(16)
    ref = cpu_ref.cbc(key, iv, host(y), decrypt=True)
    ops.cbc_decrypt(y, key, iv, out=y)
    assert host(y) == ref


@pytest.mark.parametrize("off_in,off_out", [(1, 0), (0, 3), (5, 5), (8, 8)])
def test_misaligned_tensors_are_staged(gpu, off_in, off_out):
    """Byte slices at any offset work (the native API needs 16-byte alignment;
    ops stage misaligned tensors through aligned temporaries)."""
    key, ctr0 = os.urandom(16), os.urandom(16)
    n = 4096 * 16 + 7
    base_in, base_out = rnd(n + 64, gpu, 21), torch.zeros(n + 64, dtype=torch.uint8, device=gpu)
    x = base_in[off_in:off_in + n]
    out = base_out[off_out:off_out + n]
    ops.ctr(x, key, ctr0, out=out)
    assert host(out) == cpu_ref.ctr(key, ctr0, host(x))
    assert host(base_out[:off_out]) == bytes(off_out)  # nothing written outside the slice
    assert host(base_out[off_out + n:]) == bytes(64 - off_out)
    # in place on a misaligned slice
    y = base_in[off_in:off_in + n]
    ref = cpu_ref.ctr(key, ctr0, host(y))
    ops.ctr(y, key, ctr0, out=y)
    assert host(y) == ref
    # ECB / CBC-decrypt / XOR / fill / checksum on misaligned slices
    m = 16 * 1000
    e = rnd(m + 16, gpu, 22)[off_in:off_in + m]
    c = ops.ecb_encrypt(e, key)
    assert host(c) == cpu_ref.ecb(key, host(e))
    iv = os.urandom(16)
    dst = torch.empty(m + 16, dtype=torch.uint8, device=gpu)[off_out:off_out + m]
    ops.cbc_decrypt(e, key, iv, out=dst)
    assert host(dst) == cpu_ref.cbc(key, iv, host(e), decrypt=True)
    a, b = rnd(m + 9, gpu, 23)[off_in:off_in + m], rnd(m + 9, gpu, 24)[off_out:off_out + m]
    assert torch.equal(ops.xor(a, b), a ^ b)
    f = torch.empty(m + 9, dtype=torch.uint8, device=gpu)
    ops.fill_random_(f[off_in:off_in + m], 7)
    g = torch.empty(m, dtype=torch.uint8, device=gpu)
    ops.fill_random_(g, 7)
    assert torch.equal(f[off_in:off_in + m], g)
    assert ops.checksum(f[off_in:off_in + m]) == ops.checksum(g)


def test_partial_overlap_is_rejected(gpu):
    buf = rnd(1 << 16, gpu, 25)
    with pytest.raises(RuntimeError, match="overlap"):
        ops.ctr(buf[:4096], os.urandom(16), os.urandom(16), out=buf[16:4112])


@pytest.mark.parametrize("impl", IMPLS)
def test_deterministic_rerun(gpu, impl):
    """Run twice, compare (race detection): no kernel has
    shared mutable state, so repeated runs are bit-identical."""
    key, ctr0 = os.urandom(32), os.urandom(16)
    x = rnd(64 << 20, gpu, 26)
    y1 = ops.ctr(x, key, ctr0, impl=impl)
    y2 = ops.ctr(x, key, ctr0, impl=impl)
    assert torch.equal(y1, y2)
    e1 = ops.ecb_encrypt(x, key, impl=impl)
    e2 = ops.ecb_encrypt(x, key, impl=impl)
    assert torch.equal(e1, e2)
    assert torch.equal(ops.ecb_decrypt(e1, key), x)


def test_clock_probe_beside_a_workload(gpu):
    """The one-wave probe co-resides with a full-chip kernel and reads a sane
    shader clock (gfx950 peak 2.4 GHz)."""
    x = torch.empty(1 << 30, dtype=torch.uint8, device=gpu)
    ops.fill_random_(x, 3)
    probe = ops.clock_probe(0.01, 0.05, device=gpu)
    key, ctr0 = os.urandom(16), os.urandom(16)
    for _ in range(120):  # ~1 ms each
        ops.ctr(x, key, ctr0, out=x)
    torch.cuda.synchronize()
    ghz = ops.clock_ghz(probe)
    assert 0.3 < ghz < 2.6, ghz


@pytest.mark.parametrize("bits", KEYBITS)
def test_aesni_shaped_device_api(gpu, bits):
    """otc_AES_{ECB_encrypt,ECB_decrypt,CTR_encrypt} (otc_aesni.h) with AES-NI
    schedules == the AES-NI CPU baseline (reference aesni.h shapes)."""
    import ctypes
    from our_tree_amd import _native
    if not cpu_ref.aesni_supported():
        pytest.skip("no AES-NI on this CPU")
    lib = _native.require_gpu_lib()
    key = os.urandom(bits // 8)
    nonce, ivec = os.urandom(4), os.urandom(8)
    n = 16 * 3001
    x = rnd(n + 5, gpu, 30)[:n]
    y = torch.empty_like(x)
    st = ctypes.c_void_p(torch.cuda.current_stream(gpu).cuda_stream)
    es, nr = cpu_ref.aesni_schedule(key)
    ds, _ = cpu_ref.aesni_schedule(key, decrypt=True)
    u8 = _native.as_u8p
    assert lib.otc_AES_CTR_encrypt(x.data_ptr(), y.data_ptr(), u8(ivec), u8(nonce), n, u8(es), nr, st) == 0
    assert host(y) == cpu_ref.aesni_ctr(key, nonce, ivec, host(x))
    assert lib.otc_AES_ECB_encrypt(x.data_ptr(), y.data_ptr(), n, u8(es), nr, st) == 0
    assert host(y) == cpu_ref.aesni_ecb(key, host(x))
    z = torch.empty_like(x)
    assert lib.otc_AES_ECB_decrypt(y.data_ptr(), z.data_ptr(), n, u8(ds), nr, st) == 0
    assert torch.equal(z, x)


@pytest.mark.parametrize("bits", [128, 256])
def test_bitslice_launch_structures(gpu, bits):
    """The split launch of the bitsliced kernels: both CTR and ECB run a bulk
    launch compiled for full tasks plus a one-workgroup edge launch for a
    partial first / last task -- on shapes with a
    partial first task, a partial last task, both, a single partial task and
    none, out of place and in place (a task run by both launches would be
    XORed twice)."""
    g = torch.Generator().manual_seed(5)
    for n, low in ((16 * 2048 * 9 + 16 * 77 + 3, 1000), (16 * 2048 * 2, 0), (16 * 100, 2040), (16 * 2048 * 40 + 16, 5)):
        key = os.urandom(bits // 8)
        ctr0 = os.urandom(8) + low.to_bytes(8, "big")
        x = torch.randint(0, 256, (n,), dtype=torch.uint8, generator=g).to(gpu)
        y = ops.ctr(x, key, ctr0, impl="bitslice")
        torch.cuda.synchronize()
        assert ops.last_impl() == "bitslice"
        assert host(y) == cpu_ref.ctr(key, ctr0, host(x)), ("ctr", n, low)
        z = x.clone()
        ops.ctr(z, key, ctr0, out=z, impl="bitslice")
        torch.cuda.synchronize()
        assert torch.equal(z, y), ("ctr-inplace", n, low)
        m = n & ~15
        e = ops.ecb_encrypt(x[:m], key, impl="bitslice")
        torch.cuda.synchronize()
        assert host(e) == cpu_ref.ecb(key, host(x[:m])), ("ecb", m)
        w = x[:m].clone()
        ops.ecb_encrypt(w, key, out=w, impl="bitslice")
        torch.cuda.synchronize()
        assert torch.equal(w, e), ("ecb-inplace", m)


def test_auto_routing_rule(gpu):
    """impl="auto" by size (docs/PERF.md, profiles/r3/auto_impl,
    profiles/r4/ecb_split): bitsliced CTR from 2 GiB (AES-128/192) or 1 GiB
    (AES-256), the co-resident split for ECB encryption from 2 GiB (round 5,
    measured with the halves truly co-resident), T-table for everything else;
    the boundaries are exact.  "split" is explicit for ECB; CTR
    has no split (removed in round 6, profiles/r6/ctr_split_rt/), so a CTR
    "split" request takes the auto choice."""
    G = 1 << 30
    cases = [(128, "ctr", 64 * G, "bitslice"), (128, "ctr", 2 * G - 16, "ttable"), (128, "ctr", 2 * G, "bitslice"),
             (256, "ctr", 1 * G, "bitslice"), (256, "ctr", 1 * G - 16, "ttable"), (256, "ctr", 4 * G, "bitslice"),
             (192, "ctr", 2 * G, "bitslice"), (192, "ctr", 2 * G - 16, "ttable"), (192, "ctr", 1 * G, "ttable"),
             (256, "ecb", 64 * G, "split"), (128, "ecb", 2 * G, "split"), (192, "ecb", 2 * G - 16, "ttable"),
             (256, "ecb", 1 * G, "ttable"),
             (128, "ctr", 16, "ttable")]
    for bits, mode, n, want in cases:
        assert ops.pick_impl("auto", bits, mode, n) == want, (bits, mode, n)
        assert ops.pick_impl("ttable", bits, mode, n) == "ttable"
        assert ops.pick_impl("bitslice", bits, mode, n) == "bitslice"
        assert ops.pick_impl("split", bits, mode, n) == (want if mode == "ctr" else "split")
    with pytest.raises(ValueError):
        ops.pick_impl("hybrid")


@pytest.mark.parametrize("bits", [128, 192, 256])
def test_ecb_split_matches_ttable(gpu, bits):
    """The co-resident split (T-table kernel on the caller's stream, bitsliced
    kernel on the auxiliary stream, both taking 2048-block units of the whole
    buffer from a shared counter) is byte-identical to the T-table alone, out
    of place and in place: two units exactly, units plus a partial remainder
    (run by the T-table's workgroup 0), and a bulk size; under two units the
    T-table runs alone."""
    for n, want in ((64 * 2048 * 16 * 3 + 48, "split"), (2048 * 16 + 16, "ttable"), (160 << 20, "split"),
                    (2 * 2048 * 16, "split"), (2 * 2048 * 16 + 2047 * 16, "split")):
        key = os.urandom(bits // 8)
        x = torch.empty(n, dtype=torch.uint8, device=gpu)
        ops.fill_random_(x, seed=n + bits)
        t = ops.ecb_encrypt(x, key, impl="ttable")
        y = ops.ecb_encrypt(x, key, impl="split")
        assert ops.last_impl() == want, (n, ops.last_impl())
        w = x.clone()
        ops.ecb_encrypt(w, key, out=w, impl="split")
        torch.cuda.synchronize()
        assert torch.equal(y, t), (bits, n)
        assert torch.equal(w, t), (bits, n, "in place")
        S = 1 << 14
        for off in (0, (n // 2) & ~15, n - S):
            assert host(y[off:off + S]) == cpu_ref.ecb(key, host(x[off:off + S])), (bits, n, off)


@pytest.mark.parametrize("k", [4, 5, 7, 64 * 5 + 1])
def test_split_bitsliced_alone(gpu, k):
    """impl="bitslice" for the whole-buffer modes is the bitsliced claim
    kernel alone: the T-table claim kernel's counter starts full, so one
    T-table workgroup runs only the remainder past the last unit and the
    bitsliced kernel (three workgroups per CU) takes every unit.  Every split
    mode (ECB in place, ECB / CBC / CFB decryption, segment decryption) still
    equals the T-table."""
    key, iv = os.urandom(32), os.urandom(16)
    n = (k * 2048 + 300) * 16
    x = torch.empty(n, dtype=torch.uint8, device=gpu)
    ops.fill_random_(x, seed=k)
    calls = {
        "ecb": lambda x, impl: ops.ecb_encrypt(x, key, impl=impl),
        "ecb-dec": lambda x, impl: ops.ecb_decrypt(x, key, impl=impl),
        "cbc-dec": lambda x, impl: ops.cbc_decrypt(x, key, iv, impl=impl),
        "cfb-dec": lambda x, impl: ops.cfb128_decrypt(x, key, iv, impl=impl),
        "cbc-dec-seg": lambda x, impl: ops.cbc_decrypt_segments(x[:n - n % 4096], key, iv, 4096, impl=impl),
        "cfb-dec-seg": lambda x, impl: ops.cfb128_decrypt_segments(x[:n - n % 4096], key, iv, 4096, impl=impl),
    }
    for name, f in calls.items():
        t = f(x, "ttable")
        y = f(x, "bitslice")
        assert ops.last_impl() == "bitslice", name
        torch.cuda.synchronize()
        assert torch.equal(y, t), (name, k)
        if name == "ecb":
            w = x.clone()
            ops.ecb_encrypt(w, key, out=w, impl="bitslice")
            torch.cuda.synchronize()
            assert torch.equal(w, t), (k, "in place")


@pytest.mark.parametrize("bits", KEYBITS)
def test_segment_encrypt_matches_oracle(gpu, bits):
    """CBC / CFB128 ENCRYPTION of independent segments runs the T-table
    kernels for every impl (the row-sliced VALU kernel was retired in round
    6: engine.cpp seg_enc_run) and equals the CPU oracle: 1-block, 512-byte,
    non-power-of-two and 4 KiB segments, an IV_s carry across the low 64
    bits, in place and out of place."""
    key = os.urandom(bits // 8)
    iv0 = os.urandom(8) + (2**64 - 700).to_bytes(8, "big")
    for seg, nseg in ((16, 64 * 19 + 37), (512, 64 * 19 + 37), (528, 64 * 17 + 5), (4096, 64 * 40 + 63),
                      (4096, 64 * 8 * 12)):
        n = seg * nseg
        x = torch.empty(n, dtype=torch.uint8, device=gpu)
        ops.fill_random_(x, seed=seg ^ bits ^ nseg)
        hx = host(x)
        for name in ("cbc", "cfb"):
            f = ops.cbc_encrypt_segments if name == "cbc" else ops.cfb128_encrypt_segments
            ref = cpu_ref.cbc_segments if name == "cbc" else cpu_ref.cfb128_segments
            t = f(x, key, iv0, seg, impl="ttable")
            assert ops.last_impl() == "ttable"
            for impl in ("auto", "bitslice", "split"):
                y = f(x, key, iv0, seg, impl=impl)
                assert ops.last_impl() == "ttable", (name, seg, nseg, impl)
                assert torch.equal(y, t), (name, bits, seg, nseg, impl)
            w = x.clone()
            f(w, key, iv0, seg, out=w)
            torch.cuda.synchronize()
            assert torch.equal(w, t), (name, bits, seg, nseg, "in place")
            hy = host(t)
            for s0 in (0, nseg // 2, nseg - 4):
                lo, hi = s0 * seg, (s0 + 4) * seg
                assert hy[lo:hi] == ref(key, sh.ctr_add(iv0, s0), hx[lo:hi], seg), (name, bits, seg, s0)
    for n in (896 << 20, 4 << 30, 64 << 30):
        for impl in ("auto", "bitslice", "split"):
            assert ops.pick_impl(impl, 256, "seg-enc", n) == "ttable"


@pytest.mark.parametrize("seg", [512, 1024])
def test_segment_encrypt_persistent_ttable(gpu, seg):
    """Segment encryption of >= 4 GiB in segments of <= 1 KiB runs the
    persistent T-table claim kernel (64-segment units from one counter, the
    segments past the last unit in workgroup 0): two 32 MiB windows -- one
    inside the claimed units, one covering the partial last unit -- equal the
    grid kernel run on that window alone (IV iv0 + s0), sampled segments equal
    the CPU oracle, CBC and CFB, in place."""
    key = os.urandom(32)
    iv0 = os.urandom(8) + (2**64 - 3).to_bytes(8, "big")
    nseg = ((4 << 30) + 64 * 7 * seg + 5 * seg) // seg  # a partial last unit
    n = nseg * seg
    x = torch.empty(n, dtype=torch.uint8, device=gpu)
    ops.fill_random_(x, seed=seg)
    win = (32 << 20) // seg
    for name in ("cbc", "cfb"):
        f = ops.cbc_encrypt_segments if name == "cbc" else ops.cfb128_encrypt_segments
        ref = cpu_ref.cbc_segments if name == "cbc" else cpu_ref.cfb128_segments
        y = f(x, key, iv0, seg)
        assert ops.last_impl() == "ttable"
        for s0 in (nseg // 3, nseg - win):
            lo, hi = s0 * seg, (s0 + win) * seg
            g = f(x[lo:hi], key, sh.ctr_add(iv0, s0), seg)
            torch.cuda.synchronize()
            assert torch.equal(g, y[lo:hi]), (name, seg, s0, "window")
        for s0 in (0, nseg // 3, nseg - 70, nseg - 4):
            lo, hi = s0 * seg, (s0 + 4) * seg
            assert host(y[lo:hi]) == ref(key, sh.ctr_add(iv0, s0), host(x[lo:hi]), seg), (name, seg, s0)
        f(x, key, iv0, seg, out=x)
        torch.cuda.synchronize()
        assert torch.equal(x, y), (name, seg, "in place")
        del y
        ops.fill_random_(x, seed=seg)


@pytest.mark.parametrize("bits", [128, 256])
def test_ctr_split_request_runs_auto(gpu, bits):
    """CTR has no split: impl "split" runs what "auto" picks (the bitsliced
    kernel from 2 GiB / 1 GiB, the T-table below) and equals the oracle."""
    key = os.urandom(bits // 8)
    ctr = os.urandom(8) + (2**64 - 2048 * 3 - 100).to_bytes(8, "big")
    n = 16 * 2048 * 9 + 16 * 37 + 5
    x = torch.empty(n, dtype=torch.uint8, device=gpu)
    ops.fill_random_(x, seed=n ^ bits)
    y = ops.ctr(x, key, ctr, impl="split")
    torch.cuda.synchronize()
    assert ops.last_impl() == "ttable"
    assert host(y) == cpu_ref.ctr(key, ctr, host(x))


@pytest.mark.parametrize("bits", [128, 256])
def test_persistent_ttable_ctr(gpu, bits):
    """CTR on the T-table from 512 MiB runs the persistent claim kernel
    (engine.cpp ctr_common, aes_tt.hip k_aes_ctr_tt_persist): byte-equal to
    the bitsliced kernel over the whole buffer and to the oracle on samples,
    with a counter that carries out of the low 64 bits inside the call, a
    counter offset that is not 4096-aligned (the virtual range's masked
    head) and a partial last block; in place too."""
    key = os.urandom(bits // 8)
    ctr = os.urandom(8) + (2**64 - 4096 * 40 - 77).to_bytes(8, "big")
    n = (600 << 20) + 16 * 2048 * 3 + 16 * 9 + 11
    x = torch.empty(n, dtype=torch.uint8, device=gpu)
    ops.fill_random_(x, seed=n ^ bits)
    y = ops.ctr(x, key, ctr, block_offset=1234567, impl="ttable")
    assert ops.last_impl() == "ttable"
    z = ops.ctr(x, key, ctr, block_offset=1234567, impl="bitslice")
    torch.cuda.synchronize()
    assert torch.equal(y, z)
    for lo in (0, n // 2 - (n // 2) % 16, n - 16 * 9 - 11):
        hi = min(n, lo + 16 * 64)
        assert host(y[lo:hi]) == cpu_ref.ctr(key, ctr, host(x[lo:hi]), 1234567 + lo // 16), lo
    ops.ctr(x, key, ctr, out=x, block_offset=1234567, impl="ttable")
    torch.cuda.synchronize()
    assert torch.equal(x, y)


def test_persistent_ttable_midsize(gpu):
    """ECB (both directions), CBC / CFB decryption and their segment forms
    between 896 MiB and 2 GiB run the persistent T-table claim kernel alone
    (engine.cpp split_form FORM_TT): equal to the bitsliced claim kernel alone
    and, on samples, to the oracle -- a size with a partial last unit, so
    workgroup 0's remainder path runs too."""
    key, iv = os.urandom(32), os.urandom(16)
    n = (960 << 20) + 16 * 2048 * 3 + 16 * 5
    x = torch.empty(n, dtype=torch.uint8, device=gpu)
    ops.fill_random_(x, seed=11)
    seg = 4096
    m = n - n % seg
    calls = {
        "ecb": (lambda i: ops.ecb_encrypt(x, key, impl=i), lambda h: cpu_ref.ecb(key, h), 0),
        "ecb-dec": (lambda i: ops.ecb_decrypt(x, key, impl=i), lambda h: cpu_ref.ecb(key, h, decrypt=True), 0),
        "cbc-dec": (lambda i: ops.cbc_decrypt(x, key, iv, impl=i), None, 0),
        "cfb-dec": (lambda i: ops.cfb128_decrypt(x, key, iv, impl=i), None, 0),
        "cbc-dec-seg": (lambda i: ops.cbc_decrypt_segments(x[:m], key, iv, seg, impl=i), None, 0),
        "cfb-dec-seg": (lambda i: ops.cfb128_decrypt_segments(x[:m], key, iv, seg, impl=i), None, 0),
    }
    for name, (f, ref, _) in calls.items():
        y = f("auto")
        assert ops.last_impl() == "ttable", name
        b = f("bitslice")
        torch.cuda.synchronize()
        assert torch.equal(y, b), name
        if ref is not None:
            for off in (0, (n // 2) & ~15, (n - 4096) & ~15):
                assert host(y[off:off + 4096]) == ref(host(x[off:off + 4096])), (name, off)
        del y, b


def test_split_after_release_resources(gpu):
    """otc_release_resources destroys the pooled split streams (both halves'
    CU-masked streams and their events); the next split builds them afresh
    and still equals the T-table."""
    from our_tree_amd import _native

    key = os.urandom(32)
    n = 16 * 2048 * 40 + 48
    x = torch.empty(n, dtype=torch.uint8, device=gpu)
    ops.fill_random_(x, seed=3)
    t = ops.ecb_encrypt(x, key, impl="ttable")
    for _ in range(2):
        y = ops.ecb_encrypt(x, key, impl="split")
        assert ops.last_impl() == "split"
        torch.cuda.synchronize()
        assert torch.equal(y, t)
        _native.require_gpu_lib().otc_release_resources()


def test_ecb_split_stream_order(gpu):
    """The caller's stream waits for BOTH kernels: work queued behind the
    split on the same stream sees the whole output, and the split starts only
    after work queued before it (fork / join events)."""
    key = os.urandom(32)
    n = 256 << 20
    x = torch.empty(n, dtype=torch.uint8, device=gpu)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        ops.fill_random_(x, seed=77)  # queued before the split on the same stream
        y = ops.ecb_encrypt(x, key, impl="split")
        z = ops.ecb_encrypt(y, key, impl="ttable")  # consumes the split's output, tail included
    s.synchronize()
    exp = cpu_ref.ecb(key, cpu_ref.ecb(key, host(x[n - 4096:])))
    assert host(z[n - 4096:]) == exp


def test_split_concurrent_calls(gpu):
    """Two splits in flight at once on two streams (each call has its own
    work counter and takes its own auxiliary stream from the pool), with ECB
    encryption, ECB / CBC / CFB decryption, equal to the T-table."""
    n = (96 << 20) + 4096 + 32
    key, iv = os.urandom(32), os.urandom(16)
    xs = [torch.empty(n, dtype=torch.uint8, device=gpu) for _ in range(2)]
    for i, x in enumerate(xs):
        ops.fill_random_(x, seed=900 + i)
    torch.cuda.synchronize()
    calls = [lambda x, impl: ops.ecb_encrypt(x, key, impl=impl), lambda x, impl: ops.ecb_decrypt(x, key, impl=impl),
             lambda x, impl: ops.cbc_decrypt(x, key, iv, impl=impl),
             lambda x, impl: ops.cfb128_decrypt(x, key, iv, impl=impl)]
    for f in calls:
        streams = [torch.cuda.Stream() for _ in xs]
        outs = []
        for x, st in zip(xs, streams):
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                outs.append(f(x, "split"))
        torch.cuda.synchronize()
        for x, y in zip(xs, outs):
            assert torch.equal(y, f(x, "ttable"))


@pytest.mark.parametrize("bits,n,want", [(128, (2 << 30) + 3, "bitslice"), (192, (2 << 30) + 3, "bitslice"),
                                         (256, (1 << 30) + 3, "bitslice")])
def test_ctr_auto_large_bitsliced(gpu, bits, n, want):
    """impl="auto" sends bulk AES CTR to the bitsliced kernel (the measured
    winner there; the call must actually run it): head, a middle window and
    the tail against the oracle, and equal to the forced T-table output."""
    key, ctr0 = os.urandom(bits // 8), os.urandom(8) + (2**64 - 12345).to_bytes(8, "big")
    x = torch.empty(n, dtype=torch.uint8, device=gpu)
    ops.fill_random_(x, seed=bits)
    y = ops.ctr(x, key, ctr0, impl="auto")
    assert ops.last_impl() == want
    t = ops.ctr(x, key, ctr0, impl="ttable")
    assert ops.last_impl() == "ttable"
    torch.cuda.synchronize()
    assert torch.equal(y, t)
    S = 1 << 16
    for off in (0, (n // 2) & ~15, n - S - 3):
        blk = off // 16
        exp = cpu_ref.ctr(key, ctr0, host(x[blk * 16:blk * 16 + S + 3]), block_offset=blk)
        assert host(y[blk * 16:blk * 16 + S + 3]) == exp
    del x, y, t
    torch.cuda.empty_cache()



@pytest.mark.parametrize("bits", [128, 192, 256])
def test_bitsliced_decrypt_matches_ttable(gpu, bits):
    """The bitsliced inverse cipher (the forward 77-LUT S-box as S^-1 = L S L,
    L o InvMixColumns o L between rounds, otc_invmix.h) and the decrypt split
    equal the T-table decryption, ECB (in and out of place) and CBC (IV on
    block 0; the split's bitsliced part takes block nt-1 as its predecessor),
    on sizes with partial first / last bitsliced tasks."""
    for n in (16 * 2048 * 9 + 16 * 77, 16 * 100, 16 * 2048 * 40 + 16, 96 << 20):
        key = os.urandom(bits // 8)
        iv = os.urandom(16)
        x = torch.empty(n, dtype=torch.uint8, device=gpu)
        ops.fill_random_(x, seed=n ^ bits)
        t = ops.ecb_decrypt(x, key, impl="ttable")
        for impl in ("bitslice", "split"):
            y = ops.ecb_decrypt(x, key, impl=impl)
            w = x.clone()
            ops.ecb_decrypt(w, key, out=w, impl=impl)
            torch.cuda.synchronize()
            assert torch.equal(y, t), ("ecb", impl, bits, n)
            assert torch.equal(w, t), ("ecb in place", impl, bits, n)
        tc = ops.cbc_decrypt(x, key, iv, impl="ttable")
        for impl in ("bitslice", "split"):
            c = ops.cbc_decrypt(x, key, iv, impl=impl)
            torch.cuda.synchronize()
            assert torch.equal(c, tc), ("cbc", impl, bits, n)
        S = min(n, 1 << 14)
        assert host(t[:S]) == cpu_ref.ecb(key, host(x[:S]), decrypt=True)
        assert host(tc[:S]) == cpu_ref.cbc(key, iv, host(x[:S]), decrypt=True)
    assert ops.pick_impl("auto", bits, "dec", 2 << 30) == "split"
    assert ops.pick_impl("auto", bits, "dec", (2 << 30) - 16) == "ttable"


@pytest.mark.parametrize("bits", [128, 192, 256])
def test_bitsliced_cfb_decrypt_matches_ttable(gpu, bits):
    """Bitsliced CFB128 decryption (the forward cipher on the input shifted one
    block back, the IV in front of block 0) and the CFB split (its bitsliced
    part enciphers block nt-1 of the input) equal the T-table kernel and the
    CPU oracle, on sizes with partial first / last bitsliced tasks, a single
    block and a size that splits."""
    for n in (16, 16 * 2048 * 9 + 16 * 77, 16 * 100, 16 * 2048 * 40 + 16, 96 << 20):
        key = os.urandom(bits // 8)
        iv = os.urandom(16)
        x = torch.empty(n, dtype=torch.uint8, device=gpu)
        ops.fill_random_(x, seed=n ^ bits ^ 7)
        t = ops.cfb128_decrypt(x, key, iv, impl="ttable")
        for impl in ("bitslice", "split"):
            y = ops.cfb128_decrypt(x, key, iv, impl=impl)
            torch.cuda.synchronize()
            assert torch.equal(y, t), ("cfb", impl, bits, n)
        w = x.clone()
        ops.cfb128_decrypt(w, key, iv, out=w, impl="bitslice")  # in place: through a copy
        torch.cuda.synchronize()
        assert torch.equal(w, t), ("cfb in place", bits, n)
        S = min(n, 1 << 14)
        assert host(t[:S]) == cpu_ref.cfb128(key, iv, host(x[:S]), decrypt=True)
        if n > S:  # the tail, with its predecessor block as the IV
            assert host(t[-S:]) == cpu_ref.cfb128(key, host(x[-S - 16:-S]), host(x[-S:]), decrypt=True)
    assert ops.pick_impl("auto", bits, "cfb-dec", 2 << 30) == "split"
    assert ops.pick_impl("auto", bits, "cfb-dec", (2 << 30) - 16) == "ttable"


@pytest.mark.parametrize("bits", [128, 256])
def test_segment_decrypt_split_matches_ttable(gpu, bits):
    """CBC / CFB128 decryption of independent segments (IV_s = iv0 + s, a
    carry across the low 64 bits of the IV included) through the claimed
    split equals the T-table kernel and the CPU oracle, for segments of 1, 32,
    256 and 4096 blocks, with a partial last unit; a non-power-of-two segment
    size runs the T-table."""
    key = os.urandom(bits // 8)
    iv0 = os.urandom(8) + (2**64 - 3).to_bytes(8, "big")
    for seg in (16, 512, 4096, 65536):
        n = 16 * 2048 * 40 + (seg if seg <= 16 * 2048 else 0) * 3
        n -= n % seg
        x = torch.empty(n, dtype=torch.uint8, device=gpu)
        ops.fill_random_(x, seed=seg ^ bits)
        for name in ("cbc", "cfb"):
            f = ops.cbc_decrypt_segments if name == "cbc" else ops.cfb128_decrypt_segments
            t = f(x, key, iv0, seg, impl="ttable")
            y = f(x, key, iv0, seg, impl="split")
            torch.cuda.synchronize()
            assert ops.last_impl() == "split", (name, seg)
            assert torch.equal(y, t), (name, bits, seg)
            hx, hy = host(x[:4 * seg]), host(y[:4 * seg])
            ref = (cpu_ref.cbc_segments(key, iv0, hx, seg, decrypt=True) if name == "cbc"
                   else cpu_ref.cfb128_segments(key, iv0, hx, seg, decrypt=True))
            assert hy == ref, (name, bits, seg)
    x = torch.empty(48 * 4096, dtype=torch.uint8, device=gpu)
    ops.fill_random_(x, seed=3)
    y = ops.cbc_decrypt_segments(x, key, iv0, 48, impl="split")
    torch.cuda.synchronize()
    assert ops.last_impl() == "ttable"
    assert host(y[:480]) == cpu_ref.cbc_segments(key, iv0, host(x[:480]), 48, decrypt=True)


@pytest.mark.parametrize("impl", ["ttable", "split"])
def test_ttable_modes_beyond_4gib(gpu, impl):
    """T-table (and claimed-split) ECB encrypt / decrypt, CBC and CFB128
    decrypt on a buffer above 4 GiB, checked against the oracle on samples at
    the head, across byte offset 2^32 (a 32-bit byte, block or unit offset
    would wrap there) and at the tail (round-3 review: no GPU test ran these
    kernels above ~3 MB)."""
    n = (4 << 30) + (1 << 20) + 48
    key = os.urandom(32)
    iv = os.urandom(16)
    x = torch.empty(n, dtype=torch.uint8, device=gpu)
    ops.fill_random_(x, seed=4242)
    S = 1 << 14
    offs = (0, (1 << 32) - S // 2, n - S)

    def check(out, f):
        torch.cuda.synchronize()
        for off in offs:
            assert host(out[off:off + S]) == f(off), off

    def prev(off):
        return iv if off == 0 else host(x[off - 16:off])

    y = ops.ecb_encrypt(x, key, impl=impl)
    check(y, lambda off: cpu_ref.ecb(key, host(x[off:off + S])))
    del y
    y = ops.ecb_decrypt(x, key, impl=impl)
    check(y, lambda off: cpu_ref.ecb(key, host(x[off:off + S]), decrypt=True))
    del y
    y = ops.cbc_decrypt(x, key, iv, impl=impl)
    check(y, lambda off: cpu_ref.cbc(key, prev(off), host(x[off:off + S]), decrypt=True))
    del y
    y = ops.cfb128_decrypt(x, key, iv, impl=impl)
    assert ops.last_impl() == impl
    check(y, lambda off: cpu_ref.cfb128(key, prev(off), host(x[off:off + S]), decrypt=True))
    del y, x
    torch.cuda.empty_cache()
