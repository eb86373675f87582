#!/usr/bin/env python3
"""Units each half of the co-resident split takes, across the process states
a caller can be in: buffer size, the caller's stream (torch's default /
null stream or a side stream), spin kernels queued on 12 other torch streams,
and a 1-rank RCCL group.  One JSON line per (state, mode).  Both halves > 0:
the T-table and bitsliced kernels ran at the same time.

Usage: python tools/coresidency_matrix.py [--out FILE]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    from our_tree_amd import _native, ops
    from our_tree_amd.parallel import dist as pdist

    torch.cuda.set_device(0)
    lib = _native.require_gpu_lib()
    outf = open(args.out, "a") if args.out else None

    def emit(rec):
        line = json.dumps(rec)
        print(line, flush=True)
        if outf:
            outf.write(line + "\n")
            outf.flush()

    emit({"runtime": _native.runtime_info()})
    x = torch.empty(8 << 30, dtype=torch.uint8, device="cuda")
    ops.fill_random_(x, seed=5)
    o = torch.empty_like(x)
    key = bytes(range(32))
    side = torch.cuda.Stream()
    busy = [torch.cuda.Stream() for _ in range(12)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    torch.cuda._sleep(5_000_000)
    torch.cuda.synchronize()
    per_s = 5_000_000 / (time.perf_counter() - t0)

    def units(mode, n, stream, spin):
        xs, os_ = x[:n], o[:n]
        if spin:
            for s in busy:
                with torch.cuda.stream(s):
                    torch.cuda._sleep(int(per_s * spin))
        fr, bk, nu = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        lib.otc_split_stats(1)
        with torch.cuda.stream(stream):
            t = time.perf_counter()
            if mode == "ecb":
                ops.ecb_encrypt(xs, key, out=os_)
            else:
                ops.cbc_decrypt(xs, key, bytes(16), out=os_)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
        lib.otc_split_last_units(ctypes.byref(fr), ctypes.byref(bk), ctypes.byref(nu))
        lib.otc_split_stats(0)
        return {"ran": ops.last_impl(), "front_bs": fr.value, "back_tt": bk.value, "units": nu.value,
                "ms_incl_sync": round(dt * 1e3, 2)}

    for nccl in (False, True):
        if nccl:
            pdist.init_from_env(force=True)
            t = torch.ones(1, device="cuda")
            torch.distributed.all_reduce(t)
            torch.cuda.synchronize()
        for gib in (2, 8):
            for sname, stream in (("null", torch.cuda.default_stream()), ("side", side)):
                for spin in (0.0, 0.002):
                    for mode in ("ecb", "cbc-dec"):
                        for rep in range(args.reps):
                            emit({"nccl": nccl, "gib": gib, "caller": sname, "spin_s": spin, "mode": mode,
                                  "rep": rep, **units(mode, gib << 30, stream, spin)})
    torch.cuda.synchronize()
    lib.otc_release_resources()
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
