"""Resume cursor of the streamed file job (our_tree_amd/parallel/filejob.py)
with the C-oracle backend: an interrupted job resumed any number of times is
byte-identical to one uninterrupted pass and to the one-shot oracle."""
import json
import os

import pytest

from our_tree_amd.models import cpu_ref
from our_tree_amd.parallel import filejob


def _mk(tmp_path, n, seed=1):
    src = tmp_path / "in.bin"
    src.write_bytes(os.urandom(n) if seed is None else bytes((i * 131 + seed) & 0xFF for i in range(n)))
    return str(src)


@pytest.mark.parametrize("mode,n", [("ctr", 10_000 * 16 + 9), ("ecb", 4096 * 16), ("cbc-dec", 3000 * 16)])
def test_interrupted_job_resumes_exactly(tmp_path, mode, n):
    key, iv = os.urandom(32), bytes([0xFF] * 15 + [0xF0])  # counter carries mid-stream
    src = _mk(tmp_path, n)
    dst = str(tmp_path / "out.bin")
    be = filejob.cpu_backend()
    chunk = 16 * 1000
    r = filejob.crypt_file(src, dst, key, iv, mode=mode, chunk_bytes=chunk, backend=be, max_chunks=2)
    assert not r["done"] and r["next_chunk"] == 2
    cur = json.load(open(dst + ".cursor"))
    assert cur["next_chunk"] == 2 and "key" not in cur and cur["bytes_done"] == 2 * chunk
    while not r["done"]:
        r = filejob.crypt_file(src, dst, key, iv, mode=mode, chunk_bytes=chunk, backend=be, max_chunks=3)
        assert r["resumed_from"] > 0
    assert not os.path.exists(dst + ".cursor")
    data = open(src, "rb").read()
    ref = {"ctr": lambda: cpu_ref.ctr(key, iv, data),
           "ecb": lambda: cpu_ref.ecb(key, data),
           "cbc-dec": lambda: cpu_ref.cbc(key, iv, data, decrypt=True)}[mode]()
    assert open(dst, "rb").read() == ref


def test_cursor_from_another_job_is_refused(tmp_path):
    src = _mk(tmp_path, 16 * 5000)
    dst = str(tmp_path / "out.bin")
    be = filejob.cpu_backend()
    filejob.crypt_file(src, dst, bytes(16), bytes(16), chunk_bytes=16 * 1000, backend=be, max_chunks=1)
    with pytest.raises(ValueError, match="different job"):
        filejob.crypt_file(src, dst, bytes([1] * 16), bytes(16), chunk_bytes=16 * 1000, backend=be)
    with pytest.raises(ValueError, match="different job"):
        filejob.crypt_file(src, dst, bytes(16), bytes(16), chunk_bytes=16 * 2000, backend=be)


def test_bad_arguments(tmp_path):
    src = _mk(tmp_path, 100)
    with pytest.raises(ValueError):
        filejob.crypt_file(src, str(tmp_path / "o"), bytes(16), mode="ecb", backend=filejob.cpu_backend())
    with pytest.raises(ValueError):
        filejob.crypt_file(src, str(tmp_path / "o"), bytes(16), chunk_bytes=100, backend=filejob.cpu_backend())


def test_empty_file(tmp_path):
    src = tmp_path / "e"
    src.write_bytes(b"")
    r = filejob.crypt_file(str(src), str(tmp_path / "o"), bytes(16), backend=filejob.cpu_backend())
    assert r["done"] and os.path.getsize(tmp_path / "o") == 0
