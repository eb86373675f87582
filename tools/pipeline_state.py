#!/usr/bin/env python3
"""Bisect the pinned pipeline's loss inside bench.py.

bench.py's pinned end-to-end row (1000 MiB AES-256 ECB through the 3-stream
pipeline) lost ~22% only when BOTH the 64 GiB headline shard had been
allocated and freed AND the RCCL scatter pass had run (profiles/r6/pipeline/).
This script recreates that process state step by step and times the pipeline
after each step, with engines / pinned buffers created at different points,
recording the per-phase event sums so the slow phase is visible.

Usage: python tools/pipeline_state.py [--gib 64] [--out FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def timed_runs(eng, pin_in, pin_out, key, iters=10) -> dict:
    eng.run("ecb", pin_in, pin_out, key)
    walls, h2d, k, d2h = [], 0.0, 0.0, 0.0
    for _ in range(iters):
        t0 = time.perf_counter()
        st = eng.run("ecb", pin_in, pin_out, key)
        walls.append(time.perf_counter() - t0)
        h2d += st["h2d_ms"] / iters
        k += st["kernel_ms"] / iters
        d2h += st["d2h_ms"] / iters
    n = pin_in.size
    wall = sum(walls) / len(walls)
    return {"gbps": round(n / wall / 1e9, 2), "gbps_min": round(n / max(walls) / 1e9, 2),
            "gbps_best": round(n / min(walls) / 1e9, 2), "h2d_ms": round(h2d, 2), "kernel_ms": round(k, 2),
            "d2h_ms": round(d2h, 2), "h2d_gbps": round(n / h2d / 1e6, 1), "d2h_gbps": round(n / d2h / 1e6, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=64)
    ap.add_argument("--mib", type=int, default=1000)
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-scatter", action="store_true")
    ap.add_argument("--no-kernel", action="store_true", help="fill the big buffer only (no CTR pass over it)")
    ap.add_argument("--keep-cache", action="store_true", help="del the big tensor without torch.cuda.empty_cache()")
    ap.add_argument("--recovery-s", type=float, default=0.0,
                    help="after the free, time 3-iteration passes back to back for this long")
    ap.add_argument("--only-big", action="store_true", help="stop after the big-buffer steps")
    args = ap.parse_args()

    from our_tree_amd import _native, ops
    from our_tree_amd.parallel import dist as pdist
    from our_tree_amd.parallel import stream as pstream

    outf = open(args.out, "a") if args.out else None

    def emit(rec):
        line = json.dumps(rec)
        print(line, flush=True)
        if outf:
            outf.write(line + "\n")
            outf.flush()

    torch.cuda.set_device(0)
    pdist.init_from_env(force=True)
    lib = _native.require_gpu_lib()
    emit({"runtime": _native.runtime_info()})
    nbytes = args.mib << 20
    rng = np.random.default_rng(1)
    key = bytes(rng.integers(0, 256, 32, dtype=np.uint8).tolist())

    def pinned_pair():
        a, b = pstream.pinned_empty(nbytes), pstream.pinned_empty(nbytes)
        a[:] = rng.integers(0, 256, nbytes, dtype=np.uint8)
        return a, b

    early_in, early_out = pinned_pair()
    early_eng = pstream.StreamEngine(0, chunk_bytes=64 << 20, depth=3)
    early_pooled = pstream.StreamEngine(0, chunk_bytes=64 << 20, depth=3, pooled_queues=True)
    emit({"step": "start", "early_engine": timed_runs(early_eng, early_in, early_out, key)})

    big = torch.empty(int(args.gib * (1 << 30)), dtype=torch.uint8, device="cuda")
    ops.fill_random_(big, seed=1)
    if not args.no_kernel:
        ops.ctr(big, key[:16], bytes(16), out=big)
    torch.cuda.synchronize()
    emit({"step": "big_resident", "early_engine": timed_runs(early_eng, early_in, early_out, key)})
    del big
    t_free = time.perf_counter()
    if not args.keep_cache:
        torch.cuda.empty_cache()
    emit({"step": "big_freed", "free_ms": round((time.perf_counter() - t_free) * 1e3, 2),
          "early_engine": timed_runs(early_eng, early_in, early_out, key)})
    while time.perf_counter() - t_free < args.recovery_s:
        emit({"step": "recovery", "t_s": round(time.perf_counter() - t_free, 3),
              "early_engine": timed_runs(early_eng, early_in, early_out, key, iters=3)})
    if args.only_big:
        early_eng.close()
        early_pooled.close()
        return

    if not args.no_scatter:
        from our_tree_amd.parallel import jobs

        sc = jobs.cbc_scatter_job(4, 512 << 20, key, bytes(range(0xA0, 0xB0)), sector=4096,
                                  device=torch.device("cuda", 0))
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        emit({"step": "scatter", "scatter_gbps": round(sc["gbps"], 1)})

    rec = {"step": "after"}
    rec["early_engine_early_pinned"] = timed_runs(early_eng, early_in, early_out, key)
    rec["early_pooled_engine"] = timed_runs(early_pooled, early_in, early_out, key)
    late_in, late_out = pinned_pair()
    rec["early_engine_late_pinned"] = timed_runs(early_eng, late_in, late_out, key)
    with pstream.StreamEngine(0, chunk_bytes=64 << 20, depth=3) as eng:
        rec["late_engine_late_pinned"] = timed_runs(eng, late_in, late_out, key)
        rec["late_engine_early_pinned"] = timed_runs(eng, early_in, early_out, key)
    emit(rec)
    # the refmethod sequence (pageable phase first) in this state
    from our_tree_amd.utils import refmethod

    r = refmethod.ecb256_three_ways(device=0)
    emit({"step": "refmethod", **{k: v for k, v in r.items() if not k.endswith("_what")}})
    early_eng.close()
    early_pooled.close()
    lib.otc_release_resources()
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
