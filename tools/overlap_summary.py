#!/usr/bin/env python3
"""Which phases of a pipelined job ran at the same time, from a rocprofv3
result database (ROCm 7 rocpd SQLite: --kernel-trace, --memory-copy-trace).

Every kernel dispatch and memory copy is an interval on the device clock;
intervals are grouped into phases by a name pattern (``--phase NAME=REGEX``,
first match wins; default: RCCL collectives, the AES kernels, H2D and D2H
copies) and, for kernels, split by the hardware queue they ran on (the
scatter and the gather of otc_multi_run strategy 1 are the same RCCL kernel
on different streams).  Prints each phase's busy time and, for every pair,
the time both were busy at once -- the overlap the pipeline was built for
(csrc/hip/pipeline.cpp: scatter(r+1) | cipher(r) | gather(r-1)).

    python3 tools/overlap_summary.py gpurun_out/trace/x_results.db [--together h2d,aes,d2h]

``--together A,B,C`` also prints the time every named phase (kernel phases
over all their queues) was busy at once: the three-stage overlap.
"""
import argparse
import re
import sqlite3
import sys
from itertools import combinations

DEFAULT = ["rccl=nccl|rccl", "aes=k_aes|k_bs", "h2d=HOST_TO_DEVICE|HtoD", "d2h=DEVICE_TO_HOST|DtoH"]


def union(iv):
    """total length covered by a list of (start, end) intervals, and the merged list"""
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return sum(e - s for s, e in out), out


def intersect(a, b):
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if e > s:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def tables(db):
    return {r[0] for r in db.execute("select name from sqlite_master where type in ('table', 'view')")}


def load(path):
    db = sqlite3.connect(f"file:{path}?mode=ro", uri=True)
    t = tables(db)
    rows = []
    if "kernels" in t:
        cols = [c[1] for c in db.execute("pragma table_info(kernels)")]
        q = "queue_id" if "queue_id" in cols else ("stream_id" if "stream_id" in cols else None)
        sel = f"select name, start, end{', ' + q if q else ''} from kernels"
        for r in db.execute(sel):
            rows.append(("kernel", r[0], int(r[1]), int(r[2]), r[3] if q else 0))
    if "memory_copies" in t:
        cols = [c[1] for c in db.execute("pragma table_info(memory_copies)")]
        name = "name" if "name" in cols else ("operation" if "operation" in cols else None)
        for r in db.execute(f"select {name}, start, end from memory_copies" if name else
                            "select 'copy', start, end from memory_copies"):
            rows.append(("copy", str(r[0]), int(r[1]), int(r[2]), 0))
    return rows


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--phase", action="append", help="NAME=REGEX (repeatable)")
    ap.add_argument("--together", default="h2d,aes,d2h", help="comma list of phases; '' to skip")
    a = ap.parse_args(argv)
    phases = [p.split("=", 1) for p in (a.phase or DEFAULT)]
    rows = load(a.db)
    if not rows:
        print(f"{a.db}: no kernel or copy records", file=sys.stderr)
        return 1
    groups = {}
    for kind, name, s, e, q in rows:
        for pname, rx in phases:
            if re.search(rx, name, re.I):
                key = f"{pname}@q{q}" if kind == "kernel" else pname
                groups.setdefault(key, []).append((s, e))
                break
    t0 = min(r[2] for r in rows)
    t1 = max(r[3] for r in rows)
    print(f"# {a.db}: {len(rows)} records over {(t1 - t0) / 1e6:.3f} ms")
    merged = {}
    print(f"{'phase':<24} {'intervals':>9} {'busy_ms':>10} {'first_ms':>9} {'last_ms':>9}")
    for k in sorted(groups):
        busy, m = union(groups[k])
        merged[k] = m
        print(f"{k:<24} {len(groups[k]):>9} {busy / 1e6:>10.3f} {(m[0][0] - t0) / 1e6:>9.3f} "
              f"{(m[-1][1] - t0) / 1e6:>9.3f}")
    print(f"\n{'overlap (both busy)':<44} {'ms':>10} {'% of smaller':>13}")
    for x, y in combinations(sorted(merged), 2):
        ov = intersect(merged[x], merged[y])
        small = min(union([tuple(i) for i in merged[x]])[0], union([tuple(i) for i in merged[y]])[0]) or 1
        print(f"{x + ' | ' + y:<44} {ov / 1e6:>10.3f} {100 * ov / small:>12.1f}%")
    names = [n for n in a.together.split(",") if n]
    if names:
        sets = []
        for n in names:
            iv = [tuple(i) for k, m in merged.items() if k.split("@")[0] == n for i in m]
            sets.append(union(iv)[1] if iv else [])
        acc = sets[0]
        for other in sets[1:]:
            acc = intersect_list(acc, other)
        both = sum(e - s for s, e in acc)
        small = min(sum(e - s for s, e in x) for x in sets) or 1
        print(f"\n{' & '.join(names) + ' (all at once)':<44} {both / 1e6:>10.3f} {100 * both / small:>12.1f}%")
    return 0


def intersect_list(a, b):
    """the intervals where both merged interval lists are busy"""
    i = j = 0
    out = []
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if e > s:
            out.append([s, e])
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


if __name__ == "__main__":
    sys.exit(main())
