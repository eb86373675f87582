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
