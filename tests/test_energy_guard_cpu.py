"""Regression guard on the headline kernel's work per byte and energy per
byte, over the committed bench records (no GPU needed).

The headline (AES-128-CTR, 64 GiB shard, the bitsliced kernel) runs at the
socket power cap, so its GB/s follows the box's held clock; two per-clock
figures do not: cycles per byte per CU at the clock the chip held during the
timed steps, and joules per GB (socket energy over the timed window,
our_tree_amd/utils/power.py).  The driver's records from round 4 on
(BENCH_rNN.json) and the builder's validation records from round 5 on
(profiles/rN/**/bench.json) must stay within 0.285 cycles/byte/CU and 0.86
J/GB each, and their median within 0.278.  The same kernel reads 0.2713
(BENCH_r04), 0.2755 (profiles/r5/validate) and 0.2816 (a round-4 builder
record) on different boxes -- the held-clock probe and the box move it by
~2-4% -- so a single record gets that much slack and the median guards the
trend.

Round 6 adds the figure at amd-smi's mean GFX clock over the energy window
(``cycles_per_byte_per_cu_at_mean_gfxclk``; derived from ``per_rank`` for older
records).  The seven r4/r5 records spread 0.2690-0.2717 on it (median 0.2701,
+-0.5%) where the probe's figure spread 0.269-0.2808, so its guard is 2% over
that median: a 2% regression in work per byte fails, box-to-box noise does
not.  The reference has no such metric: it timed wall-clock microseconds
only (/root/reference/test.c:31-40).

J/GB is a property of the box as much as of the kernel: round 6's records
read 0.786-0.816 on boxes holding 1.81-1.85 GHz and 0.847 on one holding
1.717 GHz (profiles/r6/validate_f, the same build as validate_e's 0.786), so
its per-record bound is 0.86; the per-clock figures guard the kernel."""
import glob
import json
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CYC_MAX, CYC_MEDIAN_MAX, JGB_MAX = 0.285, 0.278, 0.86
CYC_MEAN_CLK_MAX = round(0.2701 * 1.02, 4)  # 0.2755
FIRST_ROUND = 4          # driver records
FIRST_BUILDER_ROUND = 5  # profiles/rN validation records


def _bench_line(text):
    for line in text.splitlines():
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            try:
                return json.loads(line)
            except ValueError:
                continue
    return None


def records():
    out = []
    for p in sorted(glob.glob(os.path.join(ROOT, "BENCH_r*.json"))):
        m = re.search(r"BENCH_r(\d+)\.json$", p)
        if not m or int(m.group(1)) < FIRST_ROUND:
            continue
        d = json.load(open(p))
        b = _bench_line(((d.get("run") or {}).get("stdout_tail")) or "")
        if b:
            out.append((os.path.relpath(p, ROOT), b))
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "**", "bench.json"), recursive=True)):
        m = re.search(r"profiles/r(\d+)/", p)
        if not m or int(m.group(1)) < FIRST_BUILDER_ROUND:
            continue
        try:
            b = json.load(open(p))
        except ValueError:
            b = _bench_line(open(p).read())
        if isinstance(b, dict) and "metric" in b:
            out.append((os.path.relpath(p, ROOT), b))
    return out


def headline(b):
    c = b.get("config") or {}
    return (c.get("model") == "AES-128-CTR" and b.get("n_gpus") == 1 and c.get("per_gpu_bytes") == 64 << 30
            and (c.get("device") in (None, "gpu")))


def test_records_exist():
    assert any(headline(b) for _, b in records()), "no committed headline record from round 4 on"


@pytest.mark.parametrize("path,b", [r for r in records() if headline(r[1])], ids=lambda x: x if isinstance(x, str) else "")
def test_headline_cycles_and_energy_per_byte(path, b):
    cyc = b.get("cycles_per_byte_per_cu_at_held_clock")
    jgb = b.get("joules_per_gb")
    assert cyc is not None and jgb is not None, (path, "record lacks the held-clock / energy fields")
    assert cyc <= CYC_MAX, (path, cyc)
    assert jgb <= JGB_MAX, (path, jgb)


def test_headline_cycles_median():
    cyc = sorted(b["cycles_per_byte_per_cu_at_held_clock"] for _, b in records()
                 if headline(b) and b.get("cycles_per_byte_per_cu_at_held_clock") is not None)
    assert cyc
    med = cyc[len(cyc) // 2] if len(cyc) % 2 else (cyc[len(cyc) // 2 - 1] + cyc[len(cyc) // 2]) / 2
    assert med <= CYC_MEDIAN_MAX, (med, cyc)


def cycles_at_mean_gfxclk(b):
    """the record's key, or the same figure from its per-rank clock and rate"""
    v = b.get("cycles_per_byte_per_cu_at_mean_gfxclk")
    if v is not None:
        return v
    vals = [d["gfxclk_mhz_mean"] * 1e6 * 256 / (d["gbps"] * 1e9) for d in b.get("per_rank") or []
            if d.get("gfxclk_mhz_mean") and d.get("gbps")]
    return max(vals) if vals else None


@pytest.mark.parametrize("path,b", [r for r in records() if headline(r[1])], ids=lambda x: x if isinstance(x, str) else "")
def test_headline_cycles_at_mean_gfxclk(path, b):
    cyc = cycles_at_mean_gfxclk(b)
    assert cyc is not None, (path, "record lacks gfxclk_mhz_mean")
    assert cyc <= CYC_MEAN_CLK_MAX, (path, cyc)


def _round_of(path):
    m = re.search(r"(?:BENCH_r|profiles/r)(\d+)", path)
    return int(m.group(1)) if m else 0


def test_mean_gfxclk_guard_catches_2pct():
    """the guard's margin: a record 2% slower per clock than the r4/r5 median
    fails (the r4/r5 records are the pre-streaming-store kernel; round 6's
    non-temporal build reads 0.2637-0.2690, below them)"""
    base = [cycles_at_mean_gfxclk(b) for p, b in records() if headline(b) and _round_of(p) <= 5]
    base = sorted(v for v in base if v is not None)
    med = base[len(base) // 2]
    assert med * 1.021 > CYC_MEAN_CLK_MAX >= max(base)
