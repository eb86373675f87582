#!/usr/bin/env python3
"""Energy budget of the headline kernel.

Splits the measured J/GB of the bitsliced AES-128-CTR bulk kernel
(k_aes_bs_t3 <NR=10, CTR, LS=8, counter caching, full tasks only>) into
parts: the kernel's static instruction mix (the kernel is straight-line, so
the static count is the per-task count -- tools/isa_count.py) priced with
the measured energy per wave-instruction of each form
(tools/ubench/valu_energy.hip, profiles/r3/energy/summary*.txt: whole chip
at 2.39 GHz, nJ above idle), the global memory traffic, and the socket's
idle power over the run's time.

The per-form prices were taken at 2.39 GHz; under the headline kernel the
chip holds ~1.8 GHz at the power cap, where each switch costs less (lower
voltage).  So the instruction terms are reported twice: priced as measured,
and scaled by one factor that makes (instructions + memory + idle) equal the
measured socket energy -- the shares, not the absolute nJ, are the budget.

    python tools/energy_budget.py build/obj/hip/aes_bs.o \
        --jgb 0.808 --gbps 1702.4 --idle-w 264 [--hbm-pj-per-bit 4]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_count  # noqa: E402

LLVM = isa_count.LLVM
TASK_BYTES = 2048 * 16

# nJ per wave-instruction above idle (profiles/r3/energy/summary.txt and
# summary_2.txt; the mean where both passes measured a form)
NJ = {
    "v_xor": (0.667 + 0.656) / 2,
    "v_and_or_2in": 0.616,      # v_and_b32 / v_or_b32
    "v_bitop3_vvv": 0.840,
    "v_bitop3_vvs": 0.776,      # one SGPR / constant operand
    "v_bfi": (0.778 + 0.752) / 2,
    "v_perm": (1.033 + 1.013) / 2,
    "v_3in": 0.832,             # v_and_or / v_or3 / v_xor3 / v_lshl_or ... (v_and_or_b32 measured)
    "v_shift": 0.528,           # v_lshlrev_b32 with an inline constant
    "ds_read_b32": 2.897,
    "nop_issue": (0.064 + 0.052) / 2,  # any issued wave-instruction's front-end share (s_nop waves)
}


def classify(op: str, args: str) -> str:
    if op.startswith("v_"):
        if op.startswith("v_xor_b32"):
            return "v_xor"
        if op.startswith(("v_and_b32", "v_or_b32")):
            return "v_and_or_2in"
        if op.startswith("v_bitop3"):
            return "v_bitop3_vvs" if re.search(r"(?:^|[ ,])(?:s\d+|s\[|0x|-?\d+\b|exec|vcc)", args) else "v_bitop3_vvv"
        if op.startswith("v_bfi"):
            return "v_bfi"
        if op.startswith("v_perm"):
            return "v_perm"
        if op.startswith(("v_and_or", "v_or3", "v_xor3", "v_lshl_or", "v_and_or", "v_add3", "v_lshl_add")):
            return "v_3in"
        if op.startswith(("v_lshl", "v_lshr", "v_ashr")):
            return "v_shift"
        return "v_other"
    if op.startswith("global_load_lds") or ("global_load" in op and "lds" in args):
        return "vmem_load_lds"
    if op.startswith("global_load"):
        return "vmem_load"
    if op.startswith("global_store"):
        return "vmem_store"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "ds_read"
    if op.startswith("ds_"):
        return "ds_other"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_endpgm", "s_setprio", "s_sleep")):
        return "wait_nop"
    if op.startswith("s_"):
        return "salu"
    return "other"


def kernel_mix(obj: str, pattern: str) -> tuple[str, Counter]:
    with tempfile.TemporaryDirectory() as tmp:
        co = isa_count.code_object(obj, tmp)
        asm = subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], check=True, capture_output=True, text=True).stdout
    for f in re.split(r"\n(?=[0-9a-f]+ <)", asm):
        m = re.match(r"[0-9a-f]+ <(.*?)>:", f)
        if not m or not re.search(pattern, m.group(1)):
            continue
        mix = Counter()
        for ln in f.splitlines()[1:]:
            mm = re.match(r"\s+([a-z_0-9]+)\s*(.*?)(?://.*)?$", ln)
            if mm:
                mix[classify(mm.group(1), mm.group(2))] += 1
        return m.group(1), mix
    raise SystemExit(f"no kernel matching {pattern} in {obj}")


def budget(mix: Counter, jgb: float, gbps: float, idle_w: float, hbm_pj_per_bit: float) -> dict:
    tasks_per_gb = 1e9 / TASK_BYTES
    price = {
        "v_xor": NJ["v_xor"], "v_and_or_2in": NJ["v_and_or_2in"], "v_bitop3_vvv": NJ["v_bitop3_vvv"],
        "v_bitop3_vvs": NJ["v_bitop3_vvs"], "v_bfi": NJ["v_bfi"], "v_perm": NJ["v_perm"], "v_3in": NJ["v_3in"],
        "v_shift": NJ["v_shift"], "v_other": NJ["v_xor"],
        # an LDS read of 16 B per lane moves 4x the bytes of the measured b32 form
        "ds_read": NJ["ds_read_b32"] * 4, "ds_other": NJ["ds_read_b32"],
        "smem": NJ["nop_issue"] * 4, "salu": NJ["nop_issue"] * 2, "wait_nop": NJ["nop_issue"],
        # the vector-memory instructions' issue / address share; their bytes are the memory term
        "vmem_load": NJ["v_xor"], "vmem_load_lds": NJ["v_xor"], "vmem_store": NJ["v_xor"], "other": NJ["nop_issue"],
    }
    instr = {k: mix[k] * price[k] * 1e-9 * tasks_per_gb for k in mix}  # J/GB at the 2.39 GHz prices
    # global memory: each byte read once and written once (in place)
    mem = 2 * 8 * hbm_pj_per_bit * 1e-12 * 1e9
    idle = idle_w / (gbps * 1e9) * 1e9  # J/GB: idle W x seconds per GB
    dyn_meas = jgb - idle - mem
    raw = sum(instr.values())
    scale = dyn_meas / raw if raw else float("nan")
    groups = {
        "S-box LUT3s + MixColumns (v_bitop3 / xor / and-or)": ["v_bitop3_vvv", "v_bitop3_vvs", "v_xor", "v_and_or_2in", "v_3in"],
        "transposes + byte moves (v_bfi / v_perm / shifts / other VALU)": ["v_bfi", "v_perm", "v_shift", "v_other"],
        "LDS staging reads": ["ds_read", "ds_other"],
        "key-term / table scalar loads + SALU": ["smem", "salu"],
        "vector-memory issue": ["vmem_load", "vmem_load_lds", "vmem_store"],
        "waits / nops / other": ["wait_nop", "other"],
    }
    rows = []
    for g, ks in groups.items():
        n = sum(mix[k] for k in ks)
        j = sum(instr.get(k, 0.0) for k in ks)
        rows.append({"part": g, "wave_instr_per_task": n, "jgb_at_2p39ghz_prices": round(j, 4),
                     "jgb_scaled": round(j * scale, 4), "share": round(j * scale / jgb, 3)})
    rows.append({"part": f"HBM traffic (2 B moved per B, {hbm_pj_per_bit} pJ/bit)", "jgb_scaled": round(mem, 4),
                 "share": round(mem / jgb, 3)})
    rows.append({"part": f"idle / static ({idle_w} W over the run)", "jgb_scaled": round(idle, 4),
                 "share": round(idle / jgb, 3)})
    return {"measured_jgb": jgb, "gbps": gbps, "instr_scale_to_held_clock": round(scale, 3),
            "mix": dict(sorted(mix.items())), "rows": rows}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("obj")
    ap.add_argument("--kernel", default=r"k_aes_bs_t3ILi10ELi0ELi8ELb1ELb1E")
    ap.add_argument("--jgb", type=float, required=True, help="measured socket J/GB of the run")
    ap.add_argument("--gbps", type=float, required=True)
    ap.add_argument("--idle-w", type=float, default=264.0, help="idle socket W (248 and 279 on two boxes)")
    ap.add_argument("--hbm-pj-per-bit", type=float, default=4.0)
    ap.add_argument("--json", action="store_true")
    args = ap.parse_args()
    name, mix = kernel_mix(args.obj, args.kernel)
    b = budget(mix, args.jgb, args.gbps, args.idle_w, args.hbm_pj_per_bit)
    b["kernel"] = name
    if args.json:
        print(json.dumps(b))
        return
    print(f"kernel {name}")
    print("mix per task: " + ", ".join(f"{k} {v}" for k, v in b["mix"].items()))
    print(f"measured {b['measured_jgb']} J/GB at {b['gbps']} GB/s; instruction prices x {b['instr_scale_to_held_clock']}"
          " to close the budget")
    print(f"{'part':66s} {'instr/task':>10s} {'J/GB@2.39':>10s} {'J/GB':>8s} {'share':>6s}")
    for r in b["rows"]:
        print(f"{r['part']:66s} {r.get('wave_instr_per_task', ''):>10} {r.get('jgb_at_2p39ghz_prices', ''):>10} "
              f"{r['jgb_scaled']:>8} {r['share']:>6}")


if __name__ == "__main__":
    main()
