#!/usr/bin/env python3
"""Proxy search for a better plane basis of the bitsliced AES state.

The bitsliced kernel keeps each state byte as 8 planes in the standard
polynomial basis.  Storing instead x' = c * x (GF(2^8) product with a constant
c) keeps MixColumns exactly as cheap -- multiplication by c commutes with
xtime, and MixColumns is otherwise XORs -- and AddRoundKey folds the same way
(k' = c * k), but changes two linear layers of the S-box:

* the top layer: the 22 linear forms of the input bits that the
  Boyar-Peralta middle consumes (T1..T27, U7) become forms of x' (f M_c^-1);
* the bottom layer: the 8 outputs, forms of the 18 products M46..M63, become
  the bits of c * S(x) (M_c times the output forms).

Proxy cost = XOR2 gates of a randomised Paar greedy for each layer (best of
N restarts).  The nonlinear middle is unchanged.  Prints the best c.

    tools/basis_search.py [--restarts 20]
"""
import argparse
import random
import sys


def gmul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        a = ((a << 1) ^ (0x11B if a & 0x80 else 0)) & 0x1FF
        b >>= 1
    return r & 0xFF


def ginv(a):
    for b in range(1, 256):
        if gmul(a, b) == 1:
            return b
    raise ValueError(a)


def mat_of_mul(c):
    """8x8 GF(2) matrix (rows = output bits, as int masks over input bits)."""
    cols = [gmul(c, 1 << j) for j in range(8)]
    return [sum(((cols[j] >> i) & 1) << j for j in range(8)) for i in range(8)]


def row_times_mat(f, m):
    """row vector f (mask over the 8 coordinates y) with y = m x  ->  mask over x"""
    r = 0
    for i in range(8):
        if (f >> i) & 1:
            r ^= m[i]
    return r


TOP = [("U7k", "U7"), ("T1", "U0", "U3"), ("T2", "U0", "U5"), ("T3", "U0", "U6"), ("T4", "U3", "U5"),
       ("T5", "U4", "U6"), ("T6", "T1", "T5"), ("T7", "U1", "U2"), ("T8", "U7k", "T6"), ("T9", "U7k", "T7"),
       ("T10", "T6", "T7"), ("T11", "U1", "U5"), ("T12", "U2", "U5"), ("T13", "T3", "T4"), ("T14", "T6", "T11"),
       ("T15", "T5", "T11"), ("T16", "T5", "T12"), ("T17", "T9", "T16"), ("T18", "U3", "U7"), ("T19", "T7", "T18"),
       ("T20", "T1", "T19"), ("T21", "U6", "U7"), ("T22", "T7", "T21"), ("T23", "T2", "T22"), ("T24", "T2", "T10"),
       ("T25", "T20", "T17"), ("T26", "T3", "T16"), ("T27", "T1", "T12")]
# forms the middle reads (as AND inputs or XOR operands)
NEEDED = ["T13", "T6", "T23", "T8", "T14", "T19", "U7k", "T3", "T16", "T22", "T9", "T26", "T20", "T17", "T1",
          "T15", "T4", "T27", "T2", "T10", "T24", "T25"]
BOTTOM = """L0 M61 M62;L1 M50 M56;L2 M46 M48;L3 M47 M55;L4 M54 M58;L5 M49 M61;L6 M62 L5;L7 M46 L3;L8 M51 M59;
L9 M52 M53;L10 M53 L4;L11 M60 L2;L12 M48 M51;L13 M50 L0;L14 M52 M61;L15 M55 L1;L16 M56 L0;L17 M57 L1;L18 M58 L8;
L19 M63 L4;L20 L0 L1;L21 L1 L7;L22 L3 L12;L23 L18 L2;L24 L15 L9;L25 L6 L10;L26 L7 L9;L27 L8 L10;L28 L11 L14;
L29 L11 L17;S0 L6 L24;S1 L16 L26;S2 L19 L28;S3 L6 L21;S4 L20 L22;S5 L25 L29;S6 L13 L27;S7 L6 L23"""


def top_forms():
    env = {f"U{a}": 1 << (7 - a) for a in range(8)}  # U_a = x_{7-a}: mask over x bits
    for d in TOP:
        v = 0
        for i in d[1:]:
            v ^= env[i]
        env[d[0]] = v
    return [env[n] for n in NEEDED]


def bottom_forms():
    env = {f"M{46 + i}": 1 << i for i in range(18)}
    for item in BOTTOM.replace("\n", "").split(";"):
        n, a, b = item.split()
        env[n] = env[a] ^ env[b]
    # S_j is output bit 7-j (x7 = S0 ... x0 = S7); return masks indexed by bit i
    return [env[f"S{7 - i}"] for i in range(8)]


def paar(targets, nvars, rnd):
    """randomised Paar greedy, XOR2 count (cancellation free)"""
    ts = [set(i for i in range(nvars) if (t >> i) & 1) for t in targets]
    ts = [t for t in ts if len(t) > 1]
    nxt = nvars
    gates = 0
    while ts:
        cnt = {}
        for t in ts:
            s = sorted(t)
            for i in range(len(s)):
                for j in range(i + 1, len(s)):
                    cnt[(s[i], s[j])] = cnt.get((s[i], s[j]), 0) + 1
        best = max(cnt.values())
        pick = rnd.choice([p for p, v in cnt.items() if v == best])
        a, b = pick
        for t in ts:
            if a in t and b in t:
                t.discard(a)
                t.discard(b)
                t.add(nxt)
        nxt += 1
        gates += 1
        ts = [t for t in ts if len(t) > 1]
    return gates


def cost(forms, nvars, restarts, seed=1):
    # dedupe, drop unit forms (an input is free)
    fs = sorted({f for f in forms if f & (f - 1)})
    rnd = random.Random(seed)
    return min(paar(fs, nvars, rnd) for _ in range(restarts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--restarts", type=int, default=20)
    args = ap.parse_args()
    top = top_forms()
    bot = bottom_forms()
    res = []
    for c in range(1, 256):
        mc = mat_of_mul(c)
        minv = mat_of_mul(ginv(c))
        # x = M_{c^-1} x'  ->  form f over x becomes f M_{c^-1} over x'
        t2 = [row_times_mat(f, minv) for f in top]
        # outputs c * S:  row i of M_c combines the output forms
        b2 = []
        for i in range(8):
            v = 0
            for j in range(8):
                if (mc[i] >> j) & 1:
                    v ^= bot[j]
            b2.append(v)
        ct = cost(t2, 8, args.restarts)
        cb = cost(b2, 18, args.restarts)
        units = sum(1 for f in t2 if not f & (f - 1))
        res.append((ct + cb, ct, cb, units, c))
        print(f"c={c:3d} top {ct:3d} bottom {cb:3d} total {ct + cb:3d} (unit forms in top: {units})",
              file=sys.stderr)
    res.sort()
    print("identity:", [r for r in res if r[4] == 1])
    for r in res[:15]:
        print(f"c=0x{r[4]:02x}: total {r[0]} (top {r[1]}, bottom {r[2]}, unit top forms {r[3]})")


if __name__ == "__main__":
    main()
