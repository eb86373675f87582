#!/usr/bin/env python3
"""Run one ``bin/otbench ... --mark`` and measure the GPU's socket energy,
power, clocks and PPT residency over exactly its timed loop.

    python3 tools/power_run.py [--label L] [--gpu 0] -- ./bin/otbench --mode ecb --bits 256 --bytes 4G \
        --inplace --iters 2000 --verify --mark

otbench prints ``OTB_MARK start`` / ``OTB_MARK end`` on stderr around its
timed loop; the meter (our_tree_amd/utils/power.py, amdsmi in process) is
started / stopped on those lines.  The child is started FIRST, before this
process touches amdsmi, and nothing here initialises HIP: the meter finds the
GPU by amdsmi index, not through torch (importing torch and initialising HIP
here took longer than a 4-32 GiB otbench needs to reach its loop, so the start
line was read up to 1.3 s late and the energy window missed the loop's first
second).  Prints otbench's JSON line extended with ``power`` (joules,
avg_socket_w, ppt_residency, gfxclk_mhz_*), ``joules_per_gb`` (energy / bytes
processed in the loop) and ``window_vs_loop`` (marks wall time / the loop's
GPU time: a window that missed part of the loop reads < 0.97 and is flagged).
Exit code: otbench's.
"""
import argparse
import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    if "--" not in sys.argv:
        sys.exit("usage: power_run.py [--label L] [--gpu N] -- CMD ...")
    i = sys.argv.index("--")
    ap = argparse.ArgumentParser()
    ap.add_argument("--label", default="")
    ap.add_argument("--gpu", type=int, default=0)
    ap.add_argument("--sample-s", type=float, default=0.05)
    a = ap.parse_args(sys.argv[1:i])
    cmd = sys.argv[i + 1:]
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)

    from our_tree_amd.utils.power import PowerMeter

    meter = PowerMeter(a.gpu, sample_s=a.sample_s, torch_bdf=False)
    stats = {"available": False, "reason": "no OTB_MARK lines (run otbench with --mark)"}
    err_tail = []
    t_start = None
    marks_s = None
    for line in p.stderr:
        s = line.strip()
        if s == "OTB_MARK start":
            t_start = time.perf_counter()
            meter.start()
        elif s == "OTB_MARK end":
            stats = meter.stop()
            marks_s = time.perf_counter() - t_start if t_start else None
        else:
            err_tail.append(line)
            err_tail = err_tail[-40:]
    out = p.stdout.read()
    rc = p.wait()
    meter.close()
    sys.stderr.write("".join(err_tail))
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    if not lines:
        print(json.dumps({"label": a.label, "error": "no JSON from the command", "rc": rc, "power": stats}))
        return rc or 1
    d = json.loads(lines[-1])
    d["label"] = a.label
    d["power"] = stats
    d["marks_wall_s"] = round(marks_s, 4) if marks_s else None  # start line -> end line, as received here
    d["meter_prime_s"] = round(meter.prime_s, 3) if meter.prime_s else None
    if stats.get("available") and d.get("bytes") and d.get("iters"):
        gb = d["bytes"] * d["iters"] / 1e9
        d["joules_per_gb"] = round(stats["joules"] / gb, 4)
        loop_s = d["iters"] * d.get("ms", 0) / 1e3
        if marks_s and loop_s > 0:
            d["window_vs_loop"] = round(marks_s / loop_s, 4)
            if d["window_vs_loop"] < 0.97:
                d["window_short"] = True  # joules_per_gb undercounts; avg_socket_w / gbps stands
                print(f"power_run: window {marks_s:.3f} s < loop {loop_s:.3f} s", file=sys.stderr)
    print(json.dumps(d), flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
