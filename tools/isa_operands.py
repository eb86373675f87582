#!/usr/bin/env python3
"""Operand statistics of the AES-128 CTR bulk kernel (k_aes_bs_t3<10, 0, 8,
true, true>) in a built object: how many VALU instructions have two or three
VGPR sources in one register bank (v[n] -> bank n mod 4), how many read an
SGPR, and the runs of consecutive SGPR-reading VALU.  Read beside
tools/ubench/valu_bank.hip (what either costs on gfx950).

    tools/isa_operands.py build/obj/hip/aes_bs.o
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_count as ic  # noqa: E402


def valu_lines(obj):
    with tempfile.TemporaryDirectory() as tmp:
        co = ic.code_object(obj, tmp)
        asm = subprocess.run([f"{ic.LLVM}/llvm-objdump", "-d", co], check=True, capture_output=True,
                             text=True).stdout
    for f in re.split(r"\n(?=[0-9a-f]+ <)", asm):
        m = re.match(r"[0-9a-f]+ <(.*?)>:", f)
        if m and "k_aes_bs_t3" in m.group(1) and re.search(r"ILi10ELi0E.*Lb1ELb1EEE", m.group(1)):
            for line in f.splitlines():
                mm = re.match(r"\s+(v_[a-z0-9_]+)\s+(.*?)(\s+//.*)?$", line)
                if mm:
                    yield mm.group(1), [a.strip().split()[0] for a in mm.group(2).split(",") if a.strip()]
            return


def main():
    banks = collections.Counter()
    n = sg = run = 0
    runs = collections.Counter()
    for op, args in valu_lines(sys.argv[1]):
        n += 1
        srcs = args[1:]
        vg = []
        for r in srcs:
            x = re.match(r"v(\d+)$", r) or re.match(r"v\[(\d+):\d+\]$", r)
            if x:
                vg.append(int(x.group(1)))
        if len(vg) >= 2:
            kind = "bitop3" if op.startswith("v_bitop3") else "other"
            banks[(kind, len(vg), len(vg) - len({v % 4 for v in vg}))] += 1
        if any(re.match(r"s\d+$|s\[", r) for r in srcs):
            sg += 1
            run += 1
        else:
            if run:
                runs[min(run, 64)] += 1
            run = 0
    print(f"VALU {n}, reading an SGPR {sg} ({sg / max(n, 1):.3f})")
    print("runs of consecutive SGPR-reading VALU (length: count, 64 = 64 or more):", dict(sorted(runs.items())))
    print("(kind, VGPR sources, sources sharing a bank beyond the first): count")
    for k, v in sorted(banks.items(), key=lambda kv: -kv[1]):
        print(f"  {k}: {v}")


if __name__ == "__main__":
    main()
