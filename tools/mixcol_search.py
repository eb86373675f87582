#!/usr/bin/env python3
"""Search a short 3-input-XOR circuit for one bitsliced AES MixColumns column
and emit it as csrc/include/otc_mixcol.h.

The column is 32 input planes a_r[i] (row r, bit i) and 32 outputs
out_r = 2 a_r ^ 3 a_{r+1} ^ a_{r+2} ^ a_{r+3}; each output is the XOR of 5 or 7
inputs.  On gfx950 a 3-input XOR is one v_bitop3_b32, so the cost of a linear
circuit is its number of XOR2/XOR3 nodes.  The straightforward forms cost 76
(d_r = a_r ^ a_{r+1} first) or 80 (the low-register t-form); a best-known XOR2
circuit has 92 gates, i.e. >= 46 XOR3.

Method: a randomised greedy in the style of Paar's algorithm, over pairs AND
triples of current signals (cancellation-free): repeatedly add the XOR that
most reduces the sum over targets of ceil((k-1)/2) (k = remaining terms),
random tie-breaking, many restarts; remaining terms are finished by XOR3
chains.  The best circuit is then list-scheduled for the fewest simultaneously
live values (each live value is a VGPR in the 3-waves-per-SIMD kernel), and
emitted in that order.

    tools/mixcol_search.py [--seeds 0:120] [--out csrc/include/otc_mixcol.h]
"""
import argparse
import itertools
import os
import random


def targets():
    def a(r, i):
        return 8 * (r % 4) + i

    def two(r, i):
        return [a(r, 7)] if i == 0 else [a(r, i - 1)] + ([a(r, 7)] if i in (1, 3, 4) else [])

    out = []
    for r in range(4):
        for i in range(8):
            s = set()
            for v in two(r, i) + two(r + 1, i) + [a(r + 1, i), a(r + 2, i), a(r + 3, i)]:
                s ^= {v}
            out.append(frozenset(s))
    return out


def joint_targets():
    """MixColumns merged with the next S-box's first layer (round 6 check):
    per output byte the forms the S-box reads -- x0 and the pairwise XORs
    x6^x5, x6^x2, x3^x1, x4^x2, x7^x4, x7^x1, x1^x0 (U7, T7, T11, T5, T4, T1,
    T3, T21 of otc_sbox_lut3.h) -- each with its own key variable (100000 + k, clear of the signal numbers),
    since every one of them is XORed with a key term."""
    mc = targets()
    out = []
    for r in range(4):
        x = [set(mc[8 * r + i]) for i in range(8)]
        for pair in ((0,), (6, 5), (6, 2), (3, 1), (4, 2), (7, 4), (7, 1), (1, 0)):
            s = set()
            for i in pair:
                s ^= x[i]
            out.append(s)
    return [frozenset(t | {100000 + k}) for k, t in enumerate(out)]


def cost(k):
    return 0 if k <= 1 else k // 2  # ceil((k - 1) / 2) XOR3 nodes


def greedy(seed, tgts=None):
    rnd = random.Random(seed)
    ts = [set(t) for t in (tgts if tgts is not None else targets())]
    nsig, prog = 32, []
    while True:
        cnt = {}
        for t in ts:
            lst = sorted(t)
            for size in (2, 3):
                for c in itertools.combinations(lst, size):
                    cnt.setdefault(c, []).append(t)
        best, bs = None, 0.0
        for c, tt in cnt.items():
            sc = sum(cost(len(t)) - cost(len(t) - (len(c) - 1)) for t in tt) - 1 + 0.5 * rnd.random()
            if sc > bs:
                best, bs = c, sc
        if best is None or bs <= 0.5:
            break
        prog.append((nsig, best))
        for t in ts:
            if all(x in t for x in best):
                t.difference_update(best)
                t.add(nsig)
        nsig += 1
    return len(prog) + sum(cost(len(t)) for t in ts), prog, ts


def dag(prog, ts):
    ops = {n: list(c) for n, c in prog}
    nxt = max([n for n, _ in prog] + [31]) + 1
    outs = []
    for t in ts:
        lst = sorted(t)
        cur, rest = lst[0], lst[1:]
        while rest:
            ops[nxt] = [cur] + rest[:2]
            cur, rest, nxt = nxt, rest[2:], nxt + 1
        outs.append(cur)
    return ops, outs


def schedule(ops, outs, seed):
    rnd = random.Random(seed)
    uses = {}
    for o in ops.values():
        for x in o:
            uses[x] = uses.get(x, 0) + 1
    keep = set(outs)
    live = {x for x in range(32) if uses.get(x, 0) or x in keep}
    done, rem, todo, order, peak = set(range(32)), dict(uses), set(ops), [], len(live)
    while todo:
        ready = [n for n in todo if all(x in done for x in ops[n])]
        n = max(ready, key=lambda n: (sum(1 for x in set(ops[n]) if rem[x] == ops[n].count(x) and x not in keep),
                                      rnd.random()))
        order.append(n)
        todo.discard(n)
        done.add(n)
        live.add(n)
        peak = max(peak, len(live))
        for x in ops[n]:
            rem[x] -= 1
            if rem[x] == 0 and x not in keep:
                live.discard(x)
    return peak, order


def emit(ops, outs, order, nops, peak, seed):
    name = {i: f"in[{i}]" for i in range(32)}
    pos = {n: k for k, n in enumerate(outs)}
    body = []
    for n in order:
        a = [name[x] for x in ops[n]]
        e = f"x3({a[0]}, {a[1]}, {a[2]})" if len(a) == 3 else f"{a[0]} ^ {a[1]}"
        if n in pos:
            body.append(f"    out[{pos[n]}] = {e};")
            name[n] = f"out[{pos[n]}]"
        else:
            body.append(f"    const W m{n} = {e};")
            name[n] = f"m{n}"
    return (
        "/* Generated by tools/mixcol_search.py -- do not edit.\n"
        f" * One bitsliced AES MixColumns column in {nops} XOR2/XOR3 nodes (v_bitop3_b32\n"
        f" * on gfx950), scheduled for a peak of {peak} live planes (greedy seed {seed}).\n"
        " * in[8r+i] = bit i of row r; out likewise; in and out must not alias. */\n"
        "#ifndef OTC_MIXCOL_H\n#define OTC_MIXCOL_H\n\nnamespace otc_bs {\n\n"
        "OTC_HD void mix_column_g(const W *in, W *out)\n{\n" + "\n".join(body) + "\n}\n\n"
        "} /* namespace otc_bs */\n\n#endif\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="0:120")
    ap.add_argument("--joint", action="store_true",
                    help="only compare MixColumns + 32 key folds with the merged first-layer targets")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "csrc",
                                                  "include", "otc_mixcol.h"))
    a = ap.parse_args()
    lo, hi = (int(x) for x in a.seeds.split(":"))
    if a.joint:
        mc = min(greedy(s)[0] for s in range(lo, hi))
        jt = min(greedy(s, joint_targets())[0] for s in range(lo, hi))
        print(f"MixColumns {mc} + 32 key-folding first-layer LUTs = {mc + 32}; merged: {jt}")
        return
    best = None
    for seed in range(lo, hi):
        nops, prog, ts = greedy(seed)
        if best is None or nops < best[0]:
            best = (nops, prog, ts, seed)
    nops, prog, ts, seed = best
    ops, outs = dag(prog, ts)
    peak, order = min((schedule(ops, outs, s) for s in range(60)), key=lambda x: x[0])
    open(a.out, "w").write(emit(ops, outs, order, nops, peak, seed))
    print(f"{nops} ops, peak {peak} (seed {seed}) -> {a.out}")


if __name__ == "__main__":
    main()
