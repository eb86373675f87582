"""Harness CLIs keep the reference's results.* output formats
(test.c:61-125, aes-modes/test.c:47-446) and the parser/summary reproduce
BASELINE.md's GB/s convention on the reference's own logs."""
import os
import re
import subprocess

import pytest

from our_tree_amd.utils import results

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


@pytest.fixture(scope="module")
def cpu_bins():
    subprocess.run(["make", "-C", ROOT, "-s", "cpu"], check=True, capture_output=True)
    return os.path.join(ROOT, "bin")


def test_rc4_harness_format(cpu_bins):
    out = subprocess.run([os.path.join(cpu_bins, "test_cpu"), "--sizes", "65536,100000", "--threads", "1,3",
                          "--iters", "4"], capture_output=True, text=True, check=True).stdout
    assert re.search(r"^RC4, 65536, 1, \nGenerated a new key in \d+, \n(\d+, ){4}\n", out, re.M)
    assert "  ARC4 test #3: passed" in out
    recs = results.parse(out)
    assert [(r["bytes"], r["threads"], len(r["us"])) for r in recs] == [(65536, 1, 4), (65536, 3, 4),
                                                                        (100000, 1, 4), (100000, 3, 4)]
    assert all(r["keygen_us"] is not None for r in recs)


def test_aes_harness_format(cpu_bins):
    out = subprocess.run([os.path.join(cpu_bins, "aes_test_cpu"), "--suite", "plain-ecb,plain-ctr,aesni-ecb,aesni-ctr",
                          "--sizes", "65536", "--threads", "1,2", "--iters", "3"], capture_output=True, text=True,
                         check=True).stdout
    recs = results.parse(out)
    labels = {r["label"] for r in recs}
    assert {"Plain ECB", "Plain CTR"} <= labels
    for r in recs:
        assert len(r["us"]) == 3


def test_default_aes_harness_is_reference_main(cpu_bins):
    out = subprocess.run([os.path.join(cpu_bins, "aes_test_cpu"), "--sizes", "16384", "--threads", "1", "--iters",
                          "2"], capture_output=True, text=True, check=True).stdout
    assert out.splitlines()[0].startswith("## CPU ")
    assert all(r["label"] == "AESNI CTR" for r in results.parse(out))


@pytest.mark.skipif(not os.path.exists(REF), reason="reference logs not mounted")
def test_parse_reference_logs_matches_baseline():
    """AES-NI CTR-256 1000MiB 8 thr = 0.519 GB/s; CUDA ECB
    1000 MiB = 2.41 GB/s (average); RC4 XOR 1000 MiB 1 thr myth = 0.252."""
    recs = results.parse(open(f"{REF}/aes-modes/results.frankchn.aesni").read())
    r = [x for x in recs if x["label"] == "AESNI CTR" and x["bytes"] == 1048576000 and x["threads"] == 8][0]
    assert abs(results.summarize(r)["gbps_median"] - 0.519) < 0.005
    g = results.parse(open(f"{REF}/aes-gpu/results.baryon").read())[-1]
    assert abs(g["bytes"] / g["average_us"] / 1e3 - 2.41) < 0.01
    m = [x for x in results.parse(open(f"{REF}/results.myth.1").read())
         if x["bytes"] == 1048576000 and x["threads"] == 1][0]
    assert abs(results.summarize(m)["gbps_median"] - 0.252) < 0.005


def test_format_roundtrip():
    txt = results.format_rc4(1024, 2, 55, [1, 2, 3]) + results.format_aes("HIP CTR", 2048, 1, [4, 5]) + \
        results.format_gpu_ecb(4096, [10, 20])
    recs = results.parse(txt)
    assert recs[0]["keygen_us"] == 55 and recs[0]["us"] == [1, 2, 3]
    assert recs[1]["label"] == "HIP CTR" and recs[2]["average_us"] == 15


@pytest.mark.parametrize("exe,args,pat", [
    ("test_o0", ["--sizes", "65536", "--threads", "1,2", "--iters", "2"], r"^RC4, 65536, 2, \n"),
    ("aes_test_o0", ["--suite", "plain-ecb,aesni-ctr", "--sizes", "65536", "--threads", "1", "--iters", "2"],
     r"^Plain ECB, 65536, 1, (\d+, ){2}\n"),
])
def test_reference_methodology_o0_build(cpu_bins, exe, args, pat):
    """bin/*_o0: the harnesses built like the reference (gcc -O0 -g -Wall
    -pedantic -std=gnu99, reference Makefile:13) print the same formats."""
    out = subprocess.run([os.path.join(cpu_bins, exe)] + args, capture_output=True, text=True, check=True).stdout
    assert re.search(pat, out, re.M), out
    assert results.parse(out)


def test_o0_build_is_unoptimised():
    """The -O0 objects really are unoptimised (DWARF producer records -O0)."""
    import glob

    objs = glob.glob(os.path.join(ROOT, "build", "obj", "o0", "*.o"))
    assert objs, "make ref-o0 produced no objects"
    r = subprocess.run(["readelf", "--debug-dump=info", os.path.join(ROOT, "build", "obj", "o0", "aes.o")],
                       capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("readelf unavailable")
    assert "-O0" in r.stdout


def test_gpu_cli_usage_errors():
    """aes_ecb_d argument errors print the reference's strings
    (main_ecb_d.cu:11-26) before touching the GPU."""
    exe = os.path.join(ROOT, "bin", "aes_ecb_d")
    if not os.path.exists(exe):
        pytest.skip("bin/aes_ecb_d not built (needs hipcc)")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and r.stdout == "USAGE: aes_ecb_d KEY PLAINTEXT [PLAINTEXT...]\n"
    r = subprocess.run([exe, "0011", "00" * 16], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and r.stdout == "Invalid AES key size.\n"
    r = subprocess.run([exe, "00" * 16, "00" * 10], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and r.stdout == "Plaintext size must be a multiple of AES block size.\n"


@pytest.mark.gpu
def test_gpu_cli_ecb_d_fips197(gpu):
    """aes_ecb_d KEYHEX CTHEX decrypts FIPS-197 C.1/C.3 on the GPU and prints
    upper-case hex (reference main_ecb_d.cu:33-37, printHexArray :62-67)."""
    exe = os.path.join(ROOT, "bin", "aes_ecb_d")
    for key, ct in (("000102030405060708090a0b0c0d0e0f", "69c4e0d86a7b0430d8cdb78070b4c55a"),
                    ("000102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f",
                     "8ea2b7ca516745bfeafc49904b496089")):
        r = subprocess.run([exe, key, ct * 2], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        assert r.stdout == "00112233445566778899AABBCCDDEEFF" * 2 + "\n"


@pytest.mark.gpu
def test_gpu_cli_ecb_e_format(gpu):
    """aes_ecb_e prints the reference's `AES ECB test, <bytes>: <us>, ...
    Average <us>` lines for its 4 sizes (main_ecb_e.cu:54-73)."""
    exe = os.path.join(ROOT, "bin", "aes_ecb_e")
    r = subprocess.run([exe, "--iters", "2"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().splitlines()
    sizes = [int(m.group(1)) for m in (re.match(r"^AES ECB test, (\d+): (\d+, ){2} Average \d+$", ln)
                                       for ln in lines) if m]
    assert sizes == [1048576, 10485760, 104857600, 1048576000], r.stdout
    recs = results.parse(r.stdout)
    assert [x["bytes"] for x in recs] == sizes and all(len(x["us"]) == 2 for x in recs)


@pytest.mark.gpu
def test_gpu_rc4_harness_rows(gpu):
    """`bin/test --device gpu`: the reference RC4 sweep (test.c:60-126,135-153)
    with GPUs as column 3 -- reference line format, every iteration timed, and
    the harness's own sampled check of out = msg ^ keystream passes (exit 0),
    followed by the ARC4 self-test lines."""
    exe = os.path.join(ROOT, "bin", "test")
    r = subprocess.run([exe, "--device", "gpu", "--sizes", "1048576,1000003", "--threads", "1", "--iters", "2"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert re.search(r"^RC4, 1048576, 1, \nGenerated a new key in \d+, \n(\d+, ){2}\n", r.stdout, re.M), r.stdout
    recs = results.parse(r.stdout)
    assert [(x["bytes"], x["threads"], len(x["us"])) for x in recs] == [(1048576, 1, 2), (1000003, 1, 2)]
    assert all(x["keygen_us"] is not None for x in recs)
    assert "  ARC4 test #3: passed" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [128, 256])
def test_gpu_aes_harness_hip_rows(gpu, bits):
    """`bin/aes_test --suite hip-ecb,hip-ctr,hip-cbc`: the aes-modes harness
    rows (aes-modes/test.c:287-350 format) on the GPU kernels, device-resident
    data; the harness checks the first 64 bytes of every GPU's shard against
    the CPU oracle after the last iteration and exits non-zero on a mismatch."""
    exe = os.path.join(ROOT, "bin", "aes_test")
    r = subprocess.run([exe, "--suite", "hip-ecb,hip-ctr,hip-cbc", "--sizes", "1048576,1048583", "--threads", "1",
                        "--iters", "2", "--bits", str(bits)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    for label in ("HIP ECB", "HIP CTR", "HIP CBC"):
        assert re.search(rf"^{label}, 1048576, 1, \d+, \d+, $", r.stdout, re.M), r.stdout
    recs = results.parse(r.stdout)
    assert sorted((x["label"], x["bytes"]) for x in recs) == sorted(
        (lb, n) for lb in ("HIP ECB", "HIP CTR", "HIP CBC") for n in (1048576, 1048583))
    assert all(x["threads"] == 1 and len(x["us"]) == 2 for x in recs)
    assert "does not match" not in r.stderr
