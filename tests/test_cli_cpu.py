"""`python -m our_tree_amd` front end on the CPU: oracle self tests and a
resumable file job through the C-oracle backend (CTR twice = identity)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    return subprocess.run([sys.executable, "-m", "our_tree_amd", *args], cwd=ROOT, capture_output=True, text=True)


def test_selftest_cpu():
    r = _run("selftest")
    assert r.returncode == 0, r.stderr
    assert all(v == 0 for v in json.loads(r.stdout.splitlines()[-1])["cpu_oracle_self_tests"].values())


def test_crypt_file_roundtrip_cpu(tmp_path):
    src, mid, back = tmp_path / "a.bin", tmp_path / "b.bin", tmp_path / "c.bin"
    data = os.urandom(100_003)
    src.write_bytes(data)
    key, iv = "11" * 32, "ff" * 15 + "f0"
    for s, d in ((src, mid), (mid, back)):
        r = _run("crypt", str(s), str(d), "--key", key, "--iv", iv, "--chunk", "16K", "--cpu")
        assert r.returncode == 0, r.stderr
        assert json.loads(r.stdout)["done"]
    assert mid.read_bytes() != data and back.read_bytes() == data


def test_bad_key_is_rejected():
    r = _run("crypt", "x", "y", "--key", "abcd", "--cpu")
    assert r.returncode == 2 and "16/24/32" in r.stderr
