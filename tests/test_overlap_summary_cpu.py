"""tools/overlap_summary.py on a synthetic rocpd-shaped database: phases,
per-queue kernel split, pairwise and all-at-once overlap."""
import os
import sqlite3
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "overlap_summary.py")


def make_db(path):
    db = sqlite3.connect(path)
    db.execute("create table kernels (name text, start int, end int, queue_id int)")
    db.execute("create table memory_copies (name text, start int, end int)")
    ms = 1_000_000
    # h2d [0,10) ms, cipher [5,15) ms, d2h [8,20) ms, RCCL on two queues
    db.execute("insert into memory_copies values ('MEMORY_COPY_HOST_TO_DEVICE', 0, ?)", (10 * ms,))
    db.execute("insert into memory_copies values ('MEMORY_COPY_DEVICE_TO_HOST', ?, ?)", (8 * ms, 20 * ms))
    db.execute("insert into kernels values ('k_aes_ctr_tt', ?, ?, 1)", (5 * ms, 15 * ms))
    db.execute("insert into kernels values ('ncclDevKernel_Scatter', 0, ?, 2)", (2 * ms,))
    db.execute("insert into kernels values ('ncclDevKernel_Gather', ?, ?, 4)", (18 * ms, 19 * ms))
    db.commit()
    db.close()


def test_overlap_numbers(tmp_path):
    p = tmp_path / "t.db"
    make_db(str(p))
    out = subprocess.run([sys.executable, TOOL, str(p)], capture_output=True, text=True, check=True).stdout
    rows = {ln[:44].strip(): ln[44:].split() for ln in out.splitlines() if "|" in ln or "all at once" in ln}
    assert rows["aes@q1 | h2d"][0] == "5.000"      # [5,10)
    assert rows["aes@q1 | d2h"][0] == "7.000"      # [8,15)
    assert rows["d2h | h2d"][0] == "2.000"         # [8,10)
    assert rows["rccl@q2 | rccl@q4"][0] == "0.000"
    assert rows["h2d & aes & d2h (all at once)"][0] == "2.000"  # [8,10)
    assert "rccl@q2" in out and "rccl@q4" in out
