"""Host sanitizers over the CPU library (race detection):
csrc/cli/san_driver.c drives the threaded bulk helpers, concurrent first use
of the lazily built AES tables and both self tests; it is built twice from
source, with ThreadSanitizer and with AddressSanitizer + UBSan, and must run
clean.  (GPU sanitizers are not available on the target pool; the kernels
have no shared mutable state -- see test_deterministic_rerun on the GPU.)"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = ["csrc/cpu/aes.c", "csrc/cpu/arc4.c", "csrc/cli/san_driver.c"]


def _build_and_run(tmp_path, flags, env_extra):
    cc = shutil.which("gcc")
    if cc is None:
        pytest.skip("gcc not available")
    exe = tmp_path / "san_driver"
    cmd = [cc, "-O1", "-g", "-std=gnu99", "-I", os.path.join(ROOT, "csrc/include"), *flags,
           *[os.path.join(ROOT, s) for s in SRCS], "-o", str(exe), "-lpthread"]
    b = subprocess.run(cmd, capture_output=True, text=True)
    if b.returncode != 0 and "cannot find" in b.stderr and "san" in b.stderr:
        pytest.skip("sanitizer runtime not installed")
    assert b.returncode == 0, b.stderr
    env = dict(os.environ, **env_extra)
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "san_driver: OK" in r.stdout
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr


def test_thread_sanitizer(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1"})


def test_address_and_ub_sanitizer(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
                   {"ASAN_OPTIONS": "detect_leaks=1"})
