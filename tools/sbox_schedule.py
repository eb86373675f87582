#!/usr/bin/env python3
"""Register-pressure scheduling of the generated LUT3 S-box.

tools/sbox_lut3.py maps the (key-folded, bottom-resynthesised) Boyar-Peralta
circuit onto 83 v_bitop3_b32 LUTs and emits them in depth-first order.
Inside the bitsliced kernel every live plane is a VGPR on top of the 120 other
state planes, and the 3-waves-per-SIMD budget is 168 VGPRs, so the S-box's
peak matters.  This post-pass re-orders the statements of
csrc/include/otc_sbox_lut3.h (any topological order computes the same
function) to minimise the peak number of simultaneously live values, by a
greedy list scheduler (prefer statements that free the most operands) with
randomised tie-breaking restarts, and appends an ``OTC_LUT_PIN(x)`` after
every statement so that a kernel can pin the order (the pins are empty
volatile asms under PIN; no instructions).

Idempotent: re-running on its own output keeps the best order found.
"""
import os
import random
import re
import sys

HDR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "csrc", "include", "otc_sbox_lut3.h")
STMT = re.compile(r"^    (?:const )?W (\w+) = (.*?);(?:\s*OTC_LUT_PIN\(\w+\);)?(\s*/\*.*\*/)?$")
TOK = re.compile(r"\b([A-Z]\w*|x\d)\b")
INPUTS = ["U%d" % i for i in range(8)]


def parse(text):
    lines = text.split("\n")
    stmts, idx = [], []
    body = next(i for i, l in enumerate(lines) if "void sbox_lut3_c(" in l)
    end = next(i for i, l in enumerate(lines) if i > body and l.strip().startswith("x7 = S0"))
    for i, l in enumerate(lines):
        if i <= body or i >= end:
            continue
        m = STMT.match(l)
        if not m or m.group(1).startswith("K") or m.group(1) in INPUTS:
            continue
        name, expr = m.group(1), m.group(2)
        deps = [t for t in TOK.findall(expr) if not t.startswith("K")]
        stmts.append((name, expr, deps, (m.group(3) or "")))
        idx.append(i)
    return lines, stmts, idx


def peak_of(order, stmts_by_name, outputs):
    uses = {}
    for n in order:
        for d in stmts_by_name[n][2]:
            uses[d] = uses.get(d, 0) + 1
    live = set(INPUTS)
    remaining = dict(uses)
    peak = len(live)
    for n in order:
        live.add(n)
        peak = max(peak, len(live))
        for d in set(stmts_by_name[n][2]):
            remaining[d] -= stmts_by_name[n][2].count(d)
            if remaining[d] == 0 and d not in outputs:
                live.discard(d)
    return peak


def schedule(stmts, outputs, seed):
    rnd = random.Random(seed)
    by = {s[0]: s for s in stmts}
    uses = {}
    for s in stmts:
        for d in s[2]:
            uses[d] = uses.get(d, 0) + 1
    remaining = dict(uses)
    done = set(INPUTS)
    order = []
    todo = set(by)
    while todo:
        ready = [n for n in todo if all(d in done for d in by[n][2])]

        def score(n):
            freed = sum(1 for d in set(by[n][2]) if remaining[d] == by[n][2].count(d) and d not in outputs)
            return (freed - 1, rnd.random())
        n = max(ready, key=score)
        order.append(n)
        todo.discard(n)
        done.add(n)
        for d in by[n][2]:
            remaining[d] -= 1
    return order


def main():
    hdr = sys.argv[1] if len(sys.argv) > 1 else HDR  # another header (e.g. an ILP run's --out)
    text = open(hdr).read()
    lines, stmts, idx = parse(text)
    by = {s[0]: s for s in stmts}
    outputs = {"S%d" % i for i in range(8)}
    cur = [s[0] for s in stmts]
    best, best_peak = cur, peak_of(cur, by, outputs)
    start_peak = best_peak
    for seed in range(4000):
        o = schedule(stmts, outputs, seed)
        p = peak_of(o, by, outputs)
        if p < best_peak:
            best, best_peak = o, p
    new = [f"    W {n} = {by[n][1]}; OTC_LUT_PIN({n});{by[n][3]}" for n in best]
    out = lines[:]
    for k, i in enumerate(idx):
        out[i] = new[k]
    open(hdr, "w").write("\n".join(out))
    print(f"peak live planes: {start_peak} -> {best_peak}", file=sys.stderr)


if __name__ == "__main__":
    main()
