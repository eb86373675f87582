#!/usr/bin/env python3
"""Per-kernel PMC summary from rocprofv3 --pmc rocpd SQLite results (ROCm 7
default output; one database per pass, several passes merged).

For each kernel whose name contains --kernel, the counters of its LAST
dispatch in every database are summed over their per-SE / per-XCD rows and
merged, then printed with derived rates:

  VALU/clk/CU    SQ_INSTS_VALU / (CUs * kernel cycles at the GRBM clock, or
                 at --ghz when no GRBM pass was given)
  per wave       instruction counts / SQ_WAVES
  wave-time      SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_VALU (x4: quad-cycles) over
                 SQ_WAVE_CYCLES
  HBM bytes      FETCH_SIZE / WRITE_SIZE (kB) per byte of payload (--bytes)

    python tools/rocpd_pmc.py --kernel bs8 --bytes 4294967296 gpurun_out/x/p*/p_results.db
"""
import argparse
import sqlite3
from collections import defaultdict


def last_dispatch_counters(path, kernel):
    db = sqlite3.connect(f"file:{path}?mode=ro", uri=True)
    rows = list(db.execute("select dispatch_id, kernel_name, counter_name, value, duration, grid_size, "
                           "workgroup_size, vgpr_count, accum_vgpr_count, lds_block_size, scratch_size "
                           "from counters_collection"))
    out = {}
    for name in sorted({r[1] for r in rows if kernel in r[1]}):
        mine = [r for r in rows if r[1] == name]
        last = max(r[0] for r in mine)
        c = defaultdict(float)
        meta = None
        for r in mine:
            if r[0] == last:
                c[r[2]] += r[3]
                meta = {"duration_ns": r[4], "grid": r[5], "wg": r[6], "vgpr": r[7], "agpr": r[8], "lds": r[9],
                        "scratch": r[10]}
        out[name] = (dict(c), meta)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("--ghz", type=float, default=0.0, help="clock for rates when no GRBM_GUI_ACTIVE pass")
    ap.add_argument("--bytes", type=float, default=0.0, help="payload bytes per dispatch (HBM bytes per byte)")
    ap.add_argument("dbs", nargs="+")
    a = ap.parse_args()
    merged = defaultdict(lambda: [{}, None])
    for p in a.dbs:
        for name, (c, meta) in last_dispatch_counters(p, a.kernel).items():
            merged[name][0].update(c)
            merged[name][1] = merged[name][1] or meta
    for name, (c, meta) in merged.items():
        print(f"== {name}")
        print(f"   dispatch {meta}")
        for k in sorted(c):
            print(f"   {k:<24} {c[k]:>18.0f}")
        dur = meta["duration_ns"] * 1e-9
        if "GRBM_GUI_ACTIVE" in c and dur > 0:
            ghz = c["GRBM_GUI_ACTIVE"] / 8 / dur / 1e9  # summed over 8 XCDs
        else:
            ghz = a.ghz
        cyc = ghz * 1e9 * dur
        if ghz:
            print(f"   clock                    {ghz:.3f} GHz over {dur * 1e3:.3f} ms")
        w = c.get("SQ_WAVES", 0)
        if "SQ_INSTS_VALU" in c and cyc:
            print(f"   VALU/clk/CU              {c['SQ_INSTS_VALU'] / a.cus / cyc:.3f}")
        if w:
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                      "SQ_INSTS_LDS"):
                if k in c:
                    print(f"   {k + ' / wave':<24} {c[k] / w:>12.1f}")
        wc = c.get("SQ_WAVE_CYCLES", 0)
        if wc:
            for k, mul in (("SQ_WAIT_INST_ANY", 1), ("SQ_WAIT_ANY", 1), ("SQ_ACTIVE_INST_ANY", 1),
                           ("SQ_ACTIVE_INST_VALU", 4)):
                if k in c:
                    print(f"   {k + ' / wave-cycles':<36} {mul * c[k] / wc:.3f}")
        if a.bytes:
            for k in ("FETCH_SIZE", "WRITE_SIZE"):
                if k in c:
                    print(f"   {k + ' per payload byte':<36} {c[k] * 1024 / a.bytes:.3f}")
        if "SQ_LDS_IDX_ACTIVE" in c and cyc:
            # LDS pipe busy per CU-cycle (a conflict-free wave64 ds_read_b32 keeps it 2 cycles)
            print(f"   LDS busy / CU-cycle                  {c['SQ_LDS_IDX_ACTIVE'] / a.cus / cyc:.3f}")
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            tot = c["TCC_HIT_sum"] + c["TCC_MISS_sum"]
            print(f"   L2 hit rate                          {c['TCC_HIT_sum'] / tot if tot else 0:.3f}")


if __name__ == "__main__":
    main()
