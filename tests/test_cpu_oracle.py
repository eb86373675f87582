"""CPU oracle: standard KATs (FIPS-197, SP 800-38A, RFC 3686, Rescorla ARC4),
differential tests against the system ``openssl`` CLI, the resumable-context
semantics of the reference API, and the bitsliced core (host build).
Mirrors the reference's self tests (aes.c:912-1330, arc4.c:124-183) plus the
differential coverage the reference never had."""
import os
import shutil
import subprocess

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from our_tree_amd.models import cpu_ref

HAVE_OPENSSL = shutil.which("openssl") is not None


def openssl(mode, key, iv, data, decrypt=False):
    cmd = ["openssl", "enc", f"-aes-{len(key) * 8}-{mode}", "-K", key.hex(), "-nopad", "-nosalt"]
    if iv is not None:
        cmd += ["-iv", iv.hex()]
    if decrypt:
        cmd.append("-d")
    return subprocess.run(cmd, input=data, capture_output=True, check=True).stdout


def py_rc4(key, n, drop=0):
    S = list(range(256))
    j = 0
    for i in range(256):
        j = (j + S[i] + key[i % len(key)]) & 255
        S[i], S[j] = S[j], S[i]
    i = j = 0
    out = bytearray()
    for _ in range(drop + n):
        i = (i + 1) & 255
        j = (j + S[i]) & 255
        S[i], S[j] = S[j], S[i]
        out.append(S[(S[i] + S[j]) & 255])
    return bytes(out[drop:])


def test_self_tests_pass():
    assert cpu_ref.self_tests(0) == {"aes": 0, "arc4": 0, "bitslice": 0}


@pytest.mark.skipif(not HAVE_OPENSSL, reason="no openssl CLI")
@pytest.mark.parametrize("bits", [128, 192, 256])
@pytest.mark.parametrize("mode", ["ecb", "cbc", "cfb", "ctr"])
def test_openssl_differential(bits, mode):
    for trial in range(3):
        key = os.urandom(bits // 8)
        iv = os.urandom(16)
        n = 16 * (1 + trial * 37) if mode in ("ecb", "cbc") else 1 + trial * 333
        data = os.urandom(n)
        ref = openssl(mode, key, None if mode == "ecb" else iv, data)
        if mode == "ecb":
            got = cpu_ref.ecb(key, data)
            assert cpu_ref.ecb(key, got, decrypt=True) == data
        elif mode == "cbc":
            got = cpu_ref.cbc(key, iv, data)
            assert cpu_ref.cbc(key, iv, got, decrypt=True) == data
        elif mode == "cfb":
            got = cpu_ref.cfb128(key, iv, data)
            assert cpu_ref.cfb128(key, iv, got, decrypt=True) == data
        else:
            got = cpu_ref.ctr(key, iv, data)
        assert got == ref


@pytest.mark.skipif(not HAVE_OPENSSL, reason="no openssl CLI")
def test_ctr_128bit_carry_matches_openssl():
    key = os.urandom(16)
    ctr = (2**64 - 2).to_bytes(16, "big")  # carry from the low into the high 64 bits
    data = os.urandom(16 * 8)
    assert cpu_ref.ctr(key, ctr, data) == openssl("ctr", key, ctr, data)
    ctr = (2**128 - 2).to_bytes(16, "big")  # full wrap
    assert cpu_ref.ctr(key, ctr, data) == openssl("ctr", key, ctr, data)


def test_ctr_resume_semantics():
    """aes_crypt_ctr's byte-granular nc_off resume (reference aes.c:869-900)."""
    key, ctr0, data = os.urandom(32), os.urandom(16), os.urandom(1000)
    whole = cpu_ref.ctr(key, ctr0, data)
    nc, sb, off = bytearray(ctr0), bytearray(16), [0]
    parts = b""
    for a, b in [(0, 7), (7, 16), (16, 50), (50, 1000)]:
        parts += cpu_ref.ctr_stream(key, nc, sb, off, data[a:b])
    assert parts == whole
    assert off[0] == 1000 % 16


@given(st.binary(min_size=1, max_size=300), st.integers(0, 2**64), st.integers(1, 8))
@settings(max_examples=60, deadline=None)
def test_ctr_threads_and_offsets(data, offset, threads):
    key, ctr0 = b"k" * 16, b"\x01" * 16
    ref = cpu_ref.ctr(key, ctr0, data, block_offset=offset)
    assert cpu_ref.ctr(key, ctr0, data, block_offset=offset, threads=threads) == ref
    # offset == stream position: encrypting a longer stream and slicing
    if offset < 100:
        longer = cpu_ref.ctr(key, ctr0, bytes(16 * offset) + data)
        assert longer[16 * offset:] == ref


def test_arc4_against_python_reference():
    for kl in (1, 5, 16, 256):
        key = os.urandom(kl)
        assert cpu_ref.arc4_keystream(key, 1000) == py_rc4(key, 1000)
        assert cpu_ref.arc4_keystream(key, 100, drop=300) == py_rc4(key, 100, drop=300)


def test_arc4_rescorla_vectors():
    ks = cpu_ref.arc4_keystream(bytes.fromhex("0123456789abcdef"), 8)
    assert cpu_ref.arc4_crypt(bytes.fromhex("0123456789abcdef"), ks).hex() == "75b7878099e0c596"


def test_rc4_h_api_is_correct_for_high_bytes():
    """The reference rc4.c overflowed on key bytes >= 0x80 (signed char
    indices); ours matches arc4 for every key byte."""
    key = bytes(range(0x80, 0x90))
    data = os.urandom(500)
    assert cpu_ref.rc4_oneshot(key, data) == cpu_ref.arc4_crypt(data, cpu_ref.arc4_keystream(key, 500))


def test_arc4_crypt_threads():
    data, ks = os.urandom(10007), os.urandom(10007)
    assert cpu_ref.arc4_crypt(data, ks, threads=7) == bytes(a ^ b for a, b in zip(data, ks))


@pytest.mark.skipif(not cpu_ref.aesni_supported(), reason="no AES-NI")
@pytest.mark.parametrize("kl", [16, 24, 32])
def test_aesni_baseline_matches_oracle(kl):
    key = os.urandom(kl)
    data = os.urandom(16 * 37 + 5)
    assert cpu_ref.aesni_ecb(key, data[: 16 * 37]) == cpu_ref.ecb(key, data[: 16 * 37])
    assert cpu_ref.aesni_ecb(key, cpu_ref.ecb(key, data[: 16 * 37]), decrypt=True) == data[: 16 * 37]
    nonce, ivec = os.urandom(4), os.urandom(8)
    block = nonce + ivec + b"\x00\x00\x00\x01"
    assert cpu_ref.aesni_ctr(key, nonce, ivec, data) == cpu_ref.ctr(key, block, data)
    # sharded (per-thread offsets) == one stream
    assert (cpu_ref.aesni_ctr(key, nonce, ivec, data[:160]) + cpu_ref.aesni_ctr(key, nonce, ivec, data[160:], 10)
            == cpu_ref.aesni_ctr(key, nonce, ivec, data))


def test_cbc_segments_semantics():
    key, iv0 = os.urandom(16), os.urandom(16)
    pt = os.urandom(64 * 5)
    ct = cpu_ref.cbc_segments(key, iv0, pt, 64)
    assert ct[64:128] == cpu_ref.cbc(key, cpu_ref.ctr128_add(iv0, 1), pt[64:128])
    assert cpu_ref.cbc_segments(key, iv0, ct, 64, decrypt=True) == pt


def test_bad_key_lengths():
    with pytest.raises(ValueError):
        cpu_ref.ecb(b"x" * 15, bytes(16))
