#!/usr/bin/env python3
"""Pin csrc/include/otc_sbox_lut3.h to the generator's output.

The shipped 77-LUT S-box body is the output of tools/sbox_choices.py (the
cover ILP, --order-seed 5, ~10 min) followed by tools/sbox_schedule.py
(minimum-live-plane statement order).  The ILP is too slow to re-run in the
test suite, so its result -- the program, in the scheduled order, plus the
generator parameters -- is recorded in tools/sbox77_cover.json, and this tool
re-emits the header body from that record:

  * every statement is parsed and evaluated on 16-variable truth tables
    (8 state bits x, 8 key bits k; the 11 key terms as sbox_key_terms() builds
    them), and the 8 outputs must equal the AES S-box of x ^ k for all 2^16
    (x, k);
  * the peak of simultaneously live planes is recomputed
    (tools/sbox_schedule.py) and must equal the recorded one;
  * the body is rendered exactly as the generators write it and, with
    --check, compared line by line with the header's body.

    tools/sbox_cover.py extract [HEADER] > tools/sbox77_cover.json   # after an ILP + schedule run
    tools/sbox_cover.py emit tools/sbox77_cover.json [HEADER] --check  # exit 1 on any difference

tests/test_sbox_cover_cpu.py runs the check (and shows that a hand edit of
the header fails it).  A future ILP run writes the record with
``tools/sbox_choices.py --order-seed N`` + ``tools/sbox_schedule.py`` +
``extract``.
"""
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import sbox_schedule  # noqa: E402

HDR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "csrc", "include", "otc_sbox_lut3.h")
NV = 16
FULL = (1 << (1 << NV)) - 1
BEGIN = "    (void)K7; (void)K03;"
END = "    x7 = S0; x6 = S1;"


def var_tt(i: int) -> int:
    """bit a of the table = bit i of the assignment a"""
    block = 1 << i
    v = ((1 << block) - 1) << block
    length = 2 * block
    while length < (1 << NV):
        v |= v << length
        length *= 2
    return v


def aes_sbox() -> list:
    def mul(a, b):
        r = 0
        while b:
            if b & 1:
                r ^= a
            a = ((a << 1) ^ 0x11B) if a & 0x80 else a << 1
            b >>= 1
        return r
    inv = [0] * 256
    for a in range(1, 256):
        for b in range(1, 256):
            if mul(a, b) == 1:
                inv[a] = b
                break
    out = []
    for a in range(256):
        b = inv[a]
        s = b ^ 0x63
        for r in range(1, 5):
            s ^= ((b << r) | (b >> (8 - r))) & 0xFF
        out.append(s)
    return out


def expected_outputs() -> dict:
    """S_j (BP numbering: x7 = S0 ... x0 = S7) as truth tables over (x, k)"""
    sb = aes_sbox()
    bits = [bytearray(1 << (NV - 3)) for _ in range(8)]
    for a in range(1 << NV):
        y = sb[(a & 0xFF) ^ (a >> 8)]
        for i in range(8):
            if (y >> i) & 1:
                bits[i][a >> 3] |= 1 << (a & 7)
    return {f"S{7 - i}": int.from_bytes(bytes(bits[i]), "little") for i in range(8)}


def inputs() -> dict:
    x = [var_tt(i) for i in range(8)]
    k = [var_tt(8 + i) for i in range(8)]
    env = {f"U{i}": x[7 - i] for i in range(8)}
    # sbox_key_terms() in otc_sbox_lut3.h: K_a belongs to U_a = x_(7-a)
    env.update(K7=k[0], K03=k[7] ^ k[4], K05=k[7] ^ k[2], K06=k[7] ^ k[1], K35=k[4] ^ k[2], K46=k[3] ^ k[1],
               K12=k[6] ^ k[5], K15=k[6] ^ k[2], K25=k[5] ^ k[2], K37=k[4] ^ k[0], K67=k[1] ^ k[0])
    return env


def lut(imm, a, b, c):
    r = 0
    for m in range(8):
        if (imm >> m) & 1:
            r |= (a if m & 4 else a ^ FULL) & (b if m & 2 else b ^ FULL) & (c if m & 1 else c ^ FULL)
    return r


LUT = re.compile(r"^lut3\((\w+), (\w+), (\w+), 0x([0-9a-fA-F]+)\)$")
BIN = re.compile(r"^(~\()?(\w+) ([\^&|]) (\w+)(\))?$")


def evaluate(stmts) -> dict:
    env = inputs()
    for name, expr in stmts:
        m = LUT.match(expr)
        if m:
            v = lut(int(m.group(4), 16), env[m.group(1)], env[m.group(2)], env[m.group(3)])
        elif BIN.match(expr):
            m = BIN.match(expr)
            a, b = env[m.group(2)], env[m.group(4)]
            v = {"^": a ^ b, "&": a & b, "|": a | b}[m.group(3)]
            if m.group(1):
                v ^= FULL
        elif re.match(r"^~\w+$", expr):
            v = env[expr[1:]] ^ FULL
        elif re.match(r"^\w+$", expr):
            v = env[expr]
        else:
            raise ValueError(f"unparsed statement {name} = {expr}")
        env[name] = v
    return env


def header_statements(text: str):
    _, stmts, _ = sbox_schedule.parse(text)
    return [(n, e) for n, e, _, _ in stmts]


def render(stmts) -> list:
    return [f"    W {n} = {e}; OTC_LUT_PIN({n});" for n, e in stmts]


def body_lines(text: str) -> list:
    lines = text.split("\n")
    a = next(i for i, ln in enumerate(lines) if ln.startswith(BEGIN))
    b = next(i for i, ln in enumerate(lines) if ln.startswith(END))
    return lines[a + 1:b]


def peak(stmts) -> int:
    by = {n: (n, e, [t for t in sbox_schedule.TOK.findall(e) if not t.startswith("K")], "") for n, e in stmts}
    return sbox_schedule.peak_of([n for n, _ in stmts], by, {f"S{i}" for i in range(8)})


def verify(cover: dict) -> list:
    """problems with the recorded program (empty list: none)"""
    stmts = [tuple(s) for s in cover["statements"]]
    errs = []
    if len(stmts) != cover["luts"]:
        errs.append(f"{len(stmts)} statements, record says {cover['luts']} LUTs")
    env = evaluate(stmts)
    exp = expected_outputs()
    for j in range(8):
        if env.get(f"S{j}") != exp[f"S{j}"]:
            errs.append(f"S{j} is not bit {7 - j} of S(x ^ k)")
    p = peak(stmts)
    if p != cover["peak_live"]:
        errs.append(f"peak of live planes {p}, record says {cover['peak_live']}")
    return errs


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    if not argv or argv[0] not in ("extract", "emit"):
        sys.exit(__doc__)
    if argv[0] == "extract":
        hdr = argv[1] if len(argv) > 1 else HDR
        stmts = header_statements(open(hdr).read())
        cover = {"generator": "tools/sbox_choices.py --order-seed 5, then tools/sbox_schedule.py "
                              "(profiles/r3/sbox77)",
                 "luts": len(stmts), "peak_live": peak(stmts), "statements": [list(s) for s in stmts]}
        errs = verify(cover)
        if errs:
            sys.exit("refusing to record a wrong program: " + "; ".join(errs))
        st = cover.pop("statements")
        print(json.dumps(cover)[:-1] + ', "statements": [\n' + ",\n".join("  " + json.dumps(x) for x in st) + "\n]}")
        return 0
    cover = json.load(open(argv[1]))
    rest = [a for a in argv[2:] if not a.startswith("--")]
    hdr = rest[0] if rest else HDR
    errs = verify(cover)
    for e in errs:
        print("cover:", e, file=sys.stderr)
    want = render([tuple(s) for s in cover["statements"]])
    if "--check" in argv:
        have = body_lines(open(hdr).read())
        if have != want:
            for i, (h, w) in enumerate(zip(have + [""] * len(want), want + [""] * len(have))):
                if h != w:
                    print(f"header body line {i + 1}: has {h.strip()!r}, generator emits {w.strip()!r}",
                          file=sys.stderr)
                    break
            return 1
    else:
        print("\n".join(want))
    return 1 if errs else 0


if __name__ == "__main__":
    sys.exit(main())
