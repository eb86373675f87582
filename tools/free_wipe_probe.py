#!/usr/bin/env python3
"""After a large hipFree, how long are host<->device copies slowed, and which
direction?  (bench.py freed its 64 GiB shard right before
the pinned pipeline row.)  Times 1000 MiB pinned D2H and H2D copies back to
back for ``--seconds`` after freeing a ``--gib`` buffer and prints one JSON
line per copy with the time since the free.

Usage: python tools/free_wipe_probe.py --gib 64 --seconds 8 [--out FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=64)
    ap.add_argument("--seconds", type=float, default=8)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    n = 1000 << 20
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    outf = open(args.out, "a") if args.out else None

    def copy_ms(d2h: bool) -> float:
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        if d2h:
            host.copy_(dev, non_blocking=True)
        else:
            dev.copy_(host, non_blocking=True)
        e.record()
        e.synchronize()
        return s.elapsed_time(e)

    def emit(rec):
        line = json.dumps(rec)
        print(line, flush=True)
        if outf:
            outf.write(line + "\n")

    for _ in range(3):
        base_d2h, base_h2d = copy_ms(True), copy_ms(False)
    emit({"phase": "before", "d2h_gbps": round(n / base_d2h / 1e6, 1), "h2d_gbps": round(n / base_h2d / 1e6, 1)})
    big = torch.empty(int(args.gib * (1 << 30)), dtype=torch.uint8, device="cuda")
    big.fill_(1)
    torch.cuda.synchronize()
    del big
    t0 = time.perf_counter()
    torch.cuda.empty_cache()
    emit({"phase": "free", "free_call_ms": round((time.perf_counter() - t0) * 1e3, 2)})
    while time.perf_counter() - t0 < args.seconds:
        d, h = copy_ms(True), copy_ms(False)
        emit({"t_s": round(time.perf_counter() - t0, 3), "d2h_gbps": round(n / d / 1e6, 1),
              "h2d_gbps": round(n / h / 1e6, 1)})


if __name__ == "__main__":
    main()
