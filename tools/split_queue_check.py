#!/usr/bin/env python3
"""Do the two halves of a claimed split co-run when the process has many
streams (torch streams, as in bench.py beside RCCL's)?  Creates N torch
streams, gives each a kernel (so its hardware queue exists), then runs the
CTR and ECB splits on one of them with split accounting on and prints the
units each side took (both > 0: co-resident) and the rate.

    python tools/split_queue_check.py [--streams 12] [--gib 8]
"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from our_tree_amd import _native, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=12)
    ap.add_argument("--gib", type=int, default=8)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    lib = _native.require_gpu_lib()
    n = a.gib << 30
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    ops.fill_random_(x, seed=7)
    streams = [torch.cuda.Stream() for _ in range(a.streams)]
    for s in streams:
        with torch.cuda.stream(s):
            x[:4096].add_(0)
    torch.cuda.synchronize()
    key16, key32, ctr = os.urandom(16), os.urandom(32), os.urandom(16)
    calls = {"ctr-128": lambda i: ops.ctr(x, key16, ctr, out=x, impl=i),
             "ctr-256": lambda i: ops.ctr(x, key32, ctr, out=x, impl=i),
             "ecb-256": lambda i: ops.ecb_encrypt(x, key32, out=x, impl=i)}
    s = streams[len(streams) // 2] if streams else torch.cuda.current_stream()
    for name, f in calls.items():
        for impl in ("split", "bitslice"):
            with torch.cuda.stream(s):
                lib.otc_split_stats(1)
                f(impl)
                torch.cuda.synchronize()
                fr, bk, nu = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
                lib.otc_split_last_units(ctypes.byref(fr), ctypes.byref(bk), ctypes.byref(nu))
                lib.otc_split_stats(0)
                f(impl)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.iters):
                    f(impl)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / a.iters
            print(json.dumps({"call": name, "impl": impl, "streams": a.streams, "gib": a.gib, "ran": ops.last_impl(),
                              "units": [fr.value, bk.value, nu.value],
                              "coresident": fr.value > 0 and bk.value > 0, "gbps": round(n / dt / 1e9, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
