#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (run_counter_collection.csv) per kernel.

For every kernel whose name matches --kernel (substring), takes the LAST
dispatch of each CSV, merges the counters of several passes (one CSV per
pass) and prints the raw values plus derived rates:

  clock            GRBM_GUI_ACTIVE / 8 XCDs / dispatch wall time
  VALU rate        SQ_INSTS_VALU (or SQ_ACTIVE_INST_VALU) / CUs / cycles
  wave-time split  SQ_ACTIVE_INST_ANY, SQ_WAIT_INST_ANY, SQ_WAIT_ANY over
                   SQ_WAVE_CYCLES (disjoint, they sum to ~1)
  per-wave counts  instruction counters / SQ_WAVES

Usage: tools/pmc_summary.py --kernel k_aes_bs gpurun_out/p1/run_counter_collection.csv [...]
"""
import argparse
import csv
import sys


def last_dispatch(path, kernel):
    rows = {}
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            if kernel not in r["Kernel_Name"]:
                continue
            rows.setdefault(int(r["Dispatch_Id"]), []).append(r)
    if not rows:
        return None
    return rows[max(rows)]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("csvs", nargs="+")
    a = ap.parse_args(argv)
    vals, meta, wall_ns = {}, None, None
    for p in a.csvs:
        rows = last_dispatch(p, a.kernel)
        if rows is None:
            print(f"{p}: no dispatch of {a.kernel}", file=sys.stderr)
            continue
        meta = rows[0]
        wall_ns = int(meta["End_Timestamp"]) - int(meta["Start_Timestamp"])
        for r in rows:
            vals[r["Counter_Name"]] = float(r["Counter_Value"])
    if meta is None:
        return 1
    print(f"kernel: {meta['Kernel_Name'][:110]}")
    print(f"  grid {meta['Grid_Size']} wg {meta['Workgroup_Size']} vgpr {meta['VGPR_Count']} "
          f"agpr {meta['Accum_VGPR_Count']} sgpr {meta['SGPR_Count']} lds {meta['LDS_Block_Size']} "
          f"scratch {meta['Scratch_Size']}")
    print(f"  profiled dispatch wall {wall_ns / 1e6:.3f} ms")
    cyc = vals.get("GRBM_GUI_ACTIVE", 0) / 8
    if cyc and wall_ns:
        print(f"  clock {cyc / wall_ns:.3f} GHz ({cyc:.4g} cycles)")
    for k in sorted(vals):
        print(f"  {k:28s} {vals[k]:.6g}")
    wc = vals.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
            if k in vals:
                print(f"  wave time {k[3:]:18s} {vals[k] / wc:.3f}")
        if cyc:
            print(f"  resident waves per CU       {4 * wc / a.cus / cyc:.2f}")
    valu = vals.get("SQ_INSTS_VALU", vals.get("SQ_ACTIVE_INST_VALU"))
    if valu and cyc:
        print(f"  VALU wave-instr / clk / CU  {valu / a.cus / cyc:.3f}  (peak 2)")
    lds = vals.get("SQ_LDS_IDX_ACTIVE")
    if lds and cyc:
        print(f"  LDS busy (IDX_ACTIVE/CU/clk) {lds / a.cus / cyc:.3f}")
        if vals.get("SQ_INSTS_LDS"):
            print(f"  LDS cycles per LDS instr    {lds / vals['SQ_INSTS_LDS']:.3f}  (2.0 = conflict-free b32)")
    waves = vals.get("SQ_WAVES")
    if waves:
        for k in sorted(vals):
            if k.startswith("SQ_INSTS") or k in ("SQ_IFETCH",):
                print(f"  per wave {k:22s} {vals[k] / waves:.1f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
