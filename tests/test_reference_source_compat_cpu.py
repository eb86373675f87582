"""Source compatibility: the reference's own harness sources --
/root/reference/test.c (RC4) and /root/reference/aes-modes/test.c (AES / AES-NI)
-- compile and link unchanged against this framework's headers (csrc/include:
arc4.h, util.h, aes.h, aesni.h) and CPU library sources, with no reference
header on the include path (the .c files are compiled from a scratch copy so
"arc4.h" resolves to ours).  The binaries are not run: their hard-wired sweeps
go up to 1000 MiB x 10 iterations; the same sweeps with our harness CLIs are
covered by tests/test_harness_cpu.py."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
INC = os.path.join(ROOT, "csrc", "include")
CPU = os.path.join(ROOT, "csrc", "cpu")

pytestmark = pytest.mark.skipif(not os.path.exists(REF), reason="reference sources not mounted")


def _build(tmp_path, ref_src, ours, extra=()):
    src = tmp_path / os.path.basename(ref_src)
    shutil.copy(ref_src, src)
    exe = tmp_path / "a.out"
    cmd = ["gcc", "-std=gnu99", "-O1", "-I", INC, str(src), *[os.path.join(CPU, f) for f in ours], *extra,
           "-lpthread", "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def _symbols(exe):
    return subprocess.run(["nm", str(exe)], capture_output=True, text=True, check=True).stdout


def test_reference_rc4_harness_builds_against_our_api(tmp_path):
    exe = _build(tmp_path, f"{REF}/test.c", ["arc4.c"])
    syms = _symbols(exe)
    for s in ("arc4_setup", "arc4_prep", "arc4_crypt", "arc4_self_test", "rc4_test"):
        assert f" {s}" in syms


def test_reference_aes_harness_builds_against_our_api(tmp_path):
    exe = _build(tmp_path, f"{REF}/aes-modes/test.c", ["aes.c", "aesni.c"], ("-maes", "-msse4.1", "-mssse3"))
    syms = _symbols(exe)
    for s in ("aes_setkey_enc", "aes_crypt_ecb", "AES_256_Key_Expansion", "AES_CTR_encrypt", "CheckAESSupport"):
        assert f" {s}" in syms
