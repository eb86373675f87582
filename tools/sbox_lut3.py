#!/usr/bin/env python3
"""Map the Boyar-Peralta AES S-box circuit onto 3-input LUTs (gfx950
v_bitop3_b32) with an exact minimum-cover ILP, and emit
csrc/include/otc_sbox_lut3.h.

Model
-----
* Primary inputs: raw state planes U0..U7 (U0 = MSB) and free "key leaves":
  K7 (the round-key mask of U7) and K_ab = K_a ^ K_b for the key-folded
  first-level XORs (computed on the scalar ALU, passed as the SGPR operand of a
  bitop3).  So the circuit computes S(x ^ k) exactly like sbox_k() in
  otc_bitslice.h.
* Every gate is a 2-input XOR/AND/XNOR (or a 3-input XOR for the key-folded
  top gates).  A LUT3 implements any node as a function of a <=3-leaf cut;
  at most ONE key leaf per LUT (gfx9 VOP3 constant-bus limit: one SGPR).
* ILP (scipy.optimize.milp / HiGHS): binary x[n,c] for every gate n and
  non-trivial cut c; each output needs exactly one cut; a selected cut requires
  every gate leaf to be implemented; minimise the number of LUTs.
* bitop3 immediate: f(0xF0, 0xCC, 0xAA) for f(src0, src1, src2) (verified
  against hipcc's own lowering of (a&b)^c and (a|b)&~c on gfx950).
* Bottom linear layer re-synthesised: BP's 38 XOR2 gates (L0..L29, S0..S7)
  compute 8 linear forms of the 18 AND outputs M46..M63; a randomised greedy
  over XOR2/XOR3 nodes with shared subexpressions (Paar-style, cancellation
  free) finds a 19-node layer, after which the ILP cover drops from 86 to 83
  LUTs.  (--bp-bottom keeps the original layer.)

Then run tools/sbox_schedule.py (statement order for the fewest live planes
+ the OTC_LUT_PIN markers).
"""
import itertools
import os
import sys

import numpy as np
from scipy.optimize import Bounds, LinearConstraint, milp

# ---- Boyar-Peralta circuit with the round key folded in --------------------
G = []  # (name, op, inputs)
def g(name, op, *ins):
    G.append((name, op, ins))

PIS = [f"U{i}" for i in range(8)] + ["K7", "K03", "K05", "K06", "K35", "K46", "K12", "K15", "K25", "K37", "K67"]
KEYS = {p for p in PIS if p.startswith("K")}

g("U7k", "xor", "U7", "K7")
g("T1", "xor", "U0", "U3", "K03"); g("T2", "xor", "U0", "U5", "K05"); g("T3", "xor", "U0", "U6", "K06")
g("T4", "xor", "U3", "U5", "K35"); g("T5", "xor", "U4", "U6", "K46")
g("T6", "xor", "T1", "T5"); g("T7", "xor", "U1", "U2", "K12"); g("T8", "xor", "U7k", "T6"); g("T9", "xor", "U7k", "T7")
g("T10", "xor", "T6", "T7"); g("T11", "xor", "U1", "U5", "K15"); g("T12", "xor", "U2", "U5", "K25")
g("T13", "xor", "T3", "T4"); g("T14", "xor", "T6", "T11"); g("T15", "xor", "T5", "T11"); g("T16", "xor", "T5", "T12")
g("T17", "xor", "T9", "T16"); g("T18", "xor", "U3", "U7", "K37"); g("T19", "xor", "T7", "T18"); g("T20", "xor", "T1", "T19")
g("T21", "xor", "U6", "U7", "K67"); g("T22", "xor", "T7", "T21"); g("T23", "xor", "T2", "T22"); g("T24", "xor", "T2", "T10")
g("T25", "xor", "T20", "T17"); g("T26", "xor", "T3", "T16"); g("T27", "xor", "T1", "T12")
M = """M1 and T13 T6;M2 and T23 T8;M3 xor T14 M1;M4 and T19 U7k;M5 xor M4 M1;M6 and T3 T16;M7 and T22 T9;
M8 xor T26 M6;M9 and T20 T17;M10 xor M9 M6;M11 and T1 T15;M12 and T4 T27;M13 xor M12 M11;M14 and T2 T10;
M15 xor M14 M11;M16 xor M3 M2;M17 xor M5 T24;M18 xor M8 M7;M19 xor M10 M15;M20 xor M16 M13;M21 xor M17 M15;
M22 xor M18 M13;M23 xor M19 T25;M24 xor M22 M23;M25 and M22 M20;M26 xor M21 M25;M27 xor M20 M21;M28 xor M23 M25;
M29 and M28 M27;M30 and M26 M24;M31 and M20 M23;M32 and M27 M31;M33 xor M27 M25;M34 and M21 M22;M35 and M24 M34;
M36 xor M24 M25;M37 xor M21 M29;M38 xor M32 M33;M39 xor M23 M30;M40 xor M35 M36;M41 xor M38 M40;M42 xor M37 M39;
M43 xor M37 M38;M44 xor M39 M40;M45 xor M42 M41;M46 and M44 T6;M47 and M40 T8;M48 and M39 U7k;M49 and M43 T16;
M50 and M38 T9;M51 and M37 T17;M52 and M42 T15;M53 and M45 T27;M54 and M41 T10;M55 and M44 T13;M56 and M40 T23;
M57 and M39 T19;M58 and M43 T3;M59 and M38 T22;M60 and M37 T20;M61 and M42 T1;M62 and M45 T4;M63 and M41 T2;
L0 xor M61 M62;L1 xor M50 M56;L2 xor M46 M48;L3 xor M47 M55;L4 xor M54 M58;L5 xor M49 M61;L6 xor M62 L5;
L7 xor M46 L3;L8 xor M51 M59;L9 xor M52 M53;L10 xor M53 L4;L11 xor M60 L2;L12 xor M48 M51;L13 xor M50 L0;
L14 xor M52 M61;L15 xor M55 L1;L16 xor M56 L0;L17 xor M57 L1;L18 xor M58 L8;L19 xor M63 L4;L20 xor L0 L1;
L21 xor L1 L7;L22 xor L3 L12;L23 xor L18 L2;L24 xor L15 L9;L25 xor L6 L10;L26 xor L7 L9;L27 xor L8 L10;
L28 xor L11 L14;L29 xor L11 L17;S0 xor L6 L24;S1 xnor L16 L26;S2 xnor L19 L28;S3 xor L6 L21;S4 xor L20 L22;
S5 xor L25 L29;S6 xnor L13 L27;S7 xnor L6 L23"""
BP_BOTTOM = "--bp-bottom" in sys.argv


def linear_form(n, gates, leaves):
    """S output as (set of leaves, complement) over the XOR/XNOR gates."""
    if n in leaves:
        return frozenset([n]), 0
    op, a, b = gates[n]
    la, ca = linear_form(a, gates, leaves)
    lb, cb = linear_form(b, gates, leaves)
    return la ^ lb, ca ^ cb ^ (1 if op == "xnor" else 0)


def bottom_greedy(forms, seed):
    """XOR2/XOR3 circuit for the linear forms; returns (nodes, remaining terms)."""
    import random
    rnd = random.Random(seed)
    cost = lambda k: 0 if k <= 1 else k // 2
    ts = [set(f) for f in forms]
    prog = []
    while True:
        cnt = {}
        for t in ts:
            for size in (2, 3):
                for c in itertools.combinations(sorted(t), size):
                    cnt.setdefault(c, []).append(t)
        best, bs = None, 0.0
        for c, tt in cnt.items():
            sc = sum(cost(len(t)) - cost(len(t) - (len(c) - 1)) for t in tt) - 1 + 0.5 * rnd.random()
            if sc > bs:
                best, bs = c, sc
        if best is None or bs <= 0.5:
            break
        name = f"B{len(prog)}"
        prog.append((name, best))
        for t in ts:
            if all(x in t for x in best):
                t.difference_update(best)
                t.add(name)
    return prog, ts


_bp = {}
for item in M.replace("\n", "").split(";"):
    n, op, a, b = item.split()
    if BP_BOTTOM or not (n.startswith("L") or n.startswith("S")):
        g(n, op, a, b)
    _bp[n] = (op, a, b)
if not BP_BOTTOM:
    leaves = {f"M{i}" for i in range(46, 64)}
    forms = [linear_form(f"S{j}", _bp, leaves) for j in range(8)]
    prog, ts = bottom_greedy([f for f, _ in forms], seed=1)
    for name, c in prog:
        g(name, "xor", *c)
    for j, t in enumerate(ts):  # each output: XOR3 chain of its remaining terms
        lst = sorted(t)
        cur, rest, k = lst[0], lst[1:], 0
        while rest:
            last = len(rest) <= 2
            name = f"S{j}" if last else f"Q{j}_{k}"
            g(name, "xnor" if (last and forms[j][1]) else "xor", cur, *rest[:2])
            cur, rest, k = name, rest[2:], k + 1
OUTS = [f"S{i}" for i in range(8)]
GATE = {n: (op, ins) for n, op, ins in G}
ORDER = [n for n, _, _ in G]


def ev(n, env, memo):
    if n in env:
        return env[n]
    if n in memo:
        return memo[n]
    op, ins = GATE[n]
    v = [ev(i, env, memo) for i in ins]
    if op == "xor":
        r = 0
        for x in v:
            r ^= x
    elif op == "xnor":
        r = 1
        for x in v:
            r ^= x
    else:
        r = v[0] & v[1]
    memo[n] = r
    return r


# ---- cut enumeration -------------------------------------------------------
K = 3
cuts = {p: [frozenset([p])] for p in PIS}
for n in ORDER:
    _, ins = GATE[n]
    acc = {frozenset()}
    for i in ins:
        nxt = set()
        for c in acc:
            for ci in cuts[i]:
                u = c | ci
                if len(u) <= K and len(u & KEYS) <= 1:
                    nxt.add(u)
        acc = nxt
    cs = set(acc)
    cuts[n] = [frozenset([n])] + sorted(cs, key=lambda c: (len(c), sorted(c)))
nontriv = {n: [c for c in cuts[n] if c != frozenset([n])] for n in ORDER}

# ---- ILP -------------------------------------------------------------------
var = [(n, c) for n in ORDER for c in nontriv[n]]
idx = {v: i for i, v in enumerate(var)}
A, lb, ub = [], [], []
for n in ORDER:  # at most one implementation per node
    row = np.zeros(len(var)); [row.__setitem__(idx[(n, c)], 1) for c in nontriv[n]]
    A.append(row); lb.append(1 if n in OUTS else 0); ub.append(1)
for (n, c) in var:  # leaf gates of a selected cut must be implemented
    for l in c:
        if l in GATE:
            row = np.zeros(len(var))
            for c2 in nontriv[l]:
                row[idx[(l, c2)]] = 1
            row[idx[(n, c)]] = -1
            A.append(row); lb.append(0); ub.append(np.inf)
res = milp(c=np.ones(len(var)), constraints=LinearConstraint(np.array(A), lb, ub), integrality=np.ones(len(var)),
           bounds=Bounds(0, 1), options={"time_limit": 600})
if res.x is None:
    sys.exit(f"ILP failed: {res.message}")
sel = {n: c for (n, c), v in zip(var, res.x) if v > 0.5}
print(f"LUT count: {len(sel)} (gates: {len(G)}), status: {res.message}", file=sys.stderr)

# ---- emit --------------------------------------------------------------------
def lut_imm(n, leaves):
    pats = [0xF0, 0xCC, 0xAA][: len(leaves)]
    imm = 0
    for bit in range(8):
        env = {l: (pats[j] >> bit) & 1 for j, l in enumerate(leaves)}
        imm |= ev(n, env, {}) << bit
    return imm

lines = []
emitted = set()
def emit(n):
    if n in emitted or n in PIS:
        return
    for l in sel[n]:
        emit(l)
    leaves = sorted(sel[n], key=lambda x: (x in KEYS, ORDER.index(x) if x in GATE else PIS.index(x)))
    # key leaf (SGPR) last = src2
    if len(leaves) == 1:
        imm = lut_imm(n, leaves)  # 1-input: identity or not
        expr = leaves[0] if (imm & 0xF0) == 0xF0 else f"~{leaves[0]}"
        lines.append(f"    const W {n} = {expr};")
    elif len(leaves) == 2:
        a, b = leaves
        tt = lut_imm(n, leaves)  # over (0xF0, 0xCC)
        f = {0x3C: f"{a} ^ {b}", 0xC3: f"~({a} ^ {b})", 0xC0: f"{a} & {b}", 0xFC: f"{a} | {b}"}.get(tt & 0xFF)
        if f is None:
            lines.append(f"    const W {n} = lut3({a}, {b}, {b}, 0x{lut_imm(n, [a, b]) :02x});  /* 2-leaf */")
        else:
            lines.append(f"    const W {n} = {f};")
    else:
        imm = lut_imm(n, leaves)
        lines.append(f"    const W {n} = lut3({leaves[0]}, {leaves[1]}, {leaves[2]}, 0x{imm:02x});")
    emitted.add(n)

for o in OUTS:
    emit(o)

hdr = f'''/*
 * otc_sbox_lut3.h -- GENERATED by tools/sbox_lut3.py (+ tools/sbox_schedule.py);
 * do not edit.
 *
 * The Boyar-Peralta AES S-box with the key folded into its inputs and its
 * bottom linear layer re-synthesised ({len(G)} gates) mapped onto {len(sel)}
 * three-input LUTs = gfx950 v_bitop3_b32 (exact minimum cover by ILP over all
 * 3-feasible cuts, <= 1 SGPR key operand per LUT).  Computes S(x ^ k) for
 * plane masks k (0 / ~0).
 */
#ifndef OTC_SBOX_LUT3_H
#define OTC_SBOX_LUT3_H

namespace otc_bs {{

/* lut3(a, b, c, imm): bit i of the result = bit (4a_i + 2b_i + c_i) of imm. */
#if defined(__HIP_DEVICE_COMPILE__)
#define lut3(a, b, c, imm) __builtin_amdgcn_bitop3_b32((a), (b), (c), (imm))
#else
static inline W lut3_host(W a, W b, W c, unsigned imm)
{{
    W r = 0;
    for (int m = 0; m < 8; ++m)
        if ((imm >> m) & 1) r |= ((m & 4) ? a : ~a) & ((m & 2) ? b : ~b) & ((m & 1) ? c : ~c);
    return r;
}}
#define lut3(a, b, c, imm) lut3_host((a), (b), (c), (imm))
#endif

/* OTC_LUT_PIN: pins each LUT output in order when PIN (no instructions;
 * statement order from tools/sbox_schedule.py, minimum peak of live planes) */
#if defined(__HIP_DEVICE_COMPILE__)
#define OTC_LUT_PIN(x) \\
    if (PIN) asm volatile("" : "+v"(x))
#else
#define OTC_LUT_PIN(x) (void)0
#endif

/* The 11 key terms the LUTs read (K7 = k0 and 10 pairwise XORs of the key
 * bit masks), in the order of sbox_lut3_c's parameters: also the layout of a
 * precomputed per-S-box key table (otc_bs::sbox_key_terms). */
#define OTC_SBOX_KEY_TERMS 11

template <int PIN = 0>
OTC_HD void sbox_lut3_c(W &x0, W &x1, W &x2, W &x3, W &x4, W &x5, W &x6, W &x7, W K7, W K03, W K05, W K06, W K35,
                        W K46, W K12, W K15, W K25, W K37, W K67)
{{
    const W U0 = x7, U1 = x6, U2 = x5, U3 = x4, U4 = x3, U5 = x2, U6 = x1, U7 = x0;
    (void)K7; (void)K03; (void)K05; (void)K06; (void)K35; (void)K46; (void)K12; (void)K15; (void)K25; (void)K37; (void)K67;
''' + "\n".join(lines) + '''
    x7 = S0; x6 = S1; x5 = S2; x4 = S3; x3 = S4; x2 = S5; x1 = S6; x0 = S7;
}

/* key terms of S(x ^ k) from the 8 plane masks k0..k7 */
OTC_HD void sbox_key_terms(W k0, W k1, W k2, W k3, W k4, W k5, W k6, W k7, W *t)
{
    t[0] = k0;      /* K7  */
    t[1] = k7 ^ k4; /* K03 */
    t[2] = k7 ^ k2; /* K05 */
    t[3] = k7 ^ k1; /* K06 */
    t[4] = k4 ^ k2; /* K35 */
    t[5] = k3 ^ k1; /* K46 */
    t[6] = k6 ^ k5; /* K12 */
    t[7] = k6 ^ k2; /* K15 */
    t[8] = k5 ^ k2; /* K25 */
    t[9] = k4 ^ k0; /* K37 */
    t[10] = k1 ^ k0; /* K67 */
}

template <int PIN = 0>
OTC_HD void sbox_lut3(W &x0, W &x1, W &x2, W &x3, W &x4, W &x5, W &x6, W &x7, W k0, W k1, W k2, W k3, W k4,
                      W k5, W k6, W k7)
{
    W t[OTC_SBOX_KEY_TERMS];
    sbox_key_terms(k0, k1, k2, k3, k4, k5, k6, k7, t);
    sbox_lut3_c<PIN>(x0, x1, x2, x3, x4, x5, x6, x7, t[0], t[1], t[2], t[3], t[4], t[5], t[6], t[7], t[8], t[9],
                     t[10]);
}

#undef lut3
#undef OTC_LUT_PIN
} /* namespace otc_bs */

#endif
'''
out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "csrc", "include", "otc_sbox_lut3.h")
open(out, "w").write(hdr)
print(f"wrote {out}", file=sys.stderr)
