#!/usr/bin/env python3
"""Per-call timeline of the co-resident split from a rocprofv3 kernel trace
(rocpd SQLite): for every T-table bulk kernel, the bitsliced bulk kernel that
ran beside it, their durations, how long both ran at once and which one ran
alone at the end -- the tail a badly chosen share leaves.

    python3 tools/split_timeline.py run_results.db [--label L]
"""
import argparse
import sqlite3
import sys


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--label", default="")
    a = ap.parse_args(argv)
    db = sqlite3.connect(f"file:{a.db}?mode=ro", uri=True)
    rows = db.execute("select name, start, end from kernels order by start").fetchall()
    # the static split's kernels, or the claimed split's (k_aes_*_tt_claim, k_aes_bs_claim)
    tt = [(s, e) for n, s, e in rows if any(k in n for k in ("k_aes_enc_tt", "k_aes_dec_tt", "_tt_claim"))]
    bsnames = [n for n, s, e in rows if "bs_claim" in n]
    bs = [(s, e) for n, s, e in rows if "k_aes_bs_t3" in n or "k_aes_bs_claim" in n]
    if not tt or not bs:
        print(f"{a.label}: no split calls (tt {len(tt)}, bs {len(bs)})")
        return 0
    out = []
    for s, e in tt:
        # the bitsliced kernel of the same call: the first that starts within the T-table's run
        mate = [b for b in bs if s - 50_000 <= b[0] <= e]
        if not mate:
            continue
        bs0, bs1 = mate[0]
        both = max(0, min(e, bs1) - max(s, bs0))
        span = max(e, bs1) - min(s, bs0)
        out.append(((e - s) / 1e6, (bs1 - bs0) / 1e6, both / 1e6, span / 1e6, "tt" if e > bs1 else "bs",
                    abs(e - bs1) / 1e6, (bs0 - s) / 1e6))
    out = out[1:] or out  # the first call is the warmup
    avg = [sum(x[i] for x in out) / len(out) for i in (0, 1, 2, 3, 5, 6)]
    last = max(set(x[4] for x in out), key=[x[4] for x in out].count)
    print(f"{a.label:28s} calls {len(out)}  tt {avg[0]:8.3f} ms  bs {avg[1]:8.3f} ms  both {avg[2]:8.3f} ms  "
          f"span {avg[3]:8.3f} ms  tail {avg[4]:7.3f} ms ({last} alone)  bs starts +{avg[5]:.3f} ms")
    return 0


if __name__ == "__main__":
    sys.exit(main())
