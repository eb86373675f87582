#!/usr/bin/env python3
"""Summarise a rocprofv3 (ROCm 7) rocpd SQLite result file as a per-kernel
table: calls, total / average / min / max device time, share, launch shape and
register / LDS / scratch footprint.

    python tools/rocpd_summary.py gpurun_out/prof/x_results.db > profiles/.../x_kernels.txt
"""
import sqlite3
import sys


def summarize(path: str) -> str:
    # read-only: a mistyped path must not create an empty database file
    db = sqlite3.connect(f"file:{path}?mode=ro", uri=True)
    rows = list(db.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
        "max(grid_x), max(workgroup_x), max(vgpr_count), max(accum_vgpr_count), max(sgpr_count), "
        "max(lds_size), max(scratch_size) from kernels group by name order by sum(duration) desc"))
    total = sum(r[2] for r in rows) or 1.0
    out = [f"# {path}: kernel dispatches (durations in microseconds, device time)",
           f"{'kernel':<96} {'calls':>5} {'total_us':>12} {'avg_us':>11} {'min_us':>11} {'max_us':>11} {'%':>6} "
           f"{'grid':>8} {'wg':>5} {'vgpr':>5} {'agpr':>5} {'sgpr':>5} {'lds':>7} {'scratch':>7}"]
    for name, n, tot, avg, mn, mx, gx, wx, vg, ag, sg, lds, scr in rows:
        out.append(f"{name[:96]:<96} {n:>5} {tot / 1e3:>12.1f} {avg / 1e3:>11.2f} {mn / 1e3:>11.2f} {mx / 1e3:>11.2f} "
                   f"{100 * tot / total:>6.2f} {gx:>8} {wx:>5} {vg:>5} {ag:>5} {sg:>5} {lds:>7} {scr:>7}")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    if len(sys.argv) < 2 or sys.argv[1] in ("-h", "--help"):
        sys.stdout.write(__doc__)
        sys.exit(0)
    for p in sys.argv[1:]:
        sys.stdout.write(summarize(p))
