#!/usr/bin/env python3
"""Serving-shaped AES-CTR: many small independent messages (own key, own
counter) on one MI355X, three ways:

  eager   one ops.ctr() launch per message (host + dispatch bound)
  graph   the same per-message launches captured once in a HIP graph
          (torch.cuda.CUDAGraph) and replayed
  batch   ops.CtrBatch: every message in ONE launch (4 KiB tiles dealt to one
          persistent workgroup per CU, per-message keys/counters from device
          descriptors)

Synthetic random messages and keys.  Prints one JSON line.

    python benchmarks/batch_ctr.py --msgs 16384 --size 4096 --keys 256
"""
import argparse
import json
import os

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # before torch / HIP: dmabuf IPC only on this host driver (as bench.py)
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from our_tree_amd import ops  # noqa: E402
from our_tree_amd.models import cpu_ref  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--msgs", type=int, default=16384)
    ap.add_argument("--size", type=int, default=4096, help="bytes per message (multiple of 16)")
    ap.add_argument("--keys", type=int, default=256)
    ap.add_argument("--bits", type=int, default=128)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--no-eager", action="store_true")
    ap.add_argument("--tile", type=int, default=None, help="blocks per tile (64/128/256; default: auto)")
    args = ap.parse_args()
    if args.size % 16:
        raise SystemExit("--size must be a multiple of 16 (messages are views of one buffer)")

    dev = torch.device("cuda", 0)
    n, size = args.msgs, args.size
    src = torch.empty(n * size, dtype=torch.uint8, device=dev)
    ops.fill_random_(src, seed=7)
    dst = torch.empty_like(src)
    xs, outs = list(src.split(size)), list(dst.split(size))
    keys = [os.urandom(args.bits // 8) for _ in range(args.keys)]
    kidx = [i % args.keys for i in range(n)]
    ctrs = [os.urandom(16) for _ in range(n)]

    def eager():
        for i in range(n):
            ops.ctr(xs[i], keys[kidx[i]], ctrs[i], out=outs[i], impl="ttable")

    res = {"metric": "AES-CTR many-message throughput", "msgs": n, "msg_bytes": size, "distinct_keys": args.keys,
           "key_bits": args.bits, "total_bytes": n * size, "data": "synthetic random messages, random keys"}
    if not args.no_eager:
        t_eager = timed(eager, 1)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            eager()
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            eager()
        t_graph = timed(g.replay, args.iters)
        res["eager"] = {"ms": round(t_eager * 1e3, 3), "msgs_per_s": round(n / t_eager), "gbps": round(n * size / t_eager / 1e9, 3)}
        res["graph"] = {"ms": round(t_graph * 1e3, 3), "msgs_per_s": round(n / t_graph), "gbps": round(n * size / t_graph / 1e9, 3)}

    t0 = time.perf_counter()
    batch = ops.CtrBatch(xs, keys, ctrs, outs=outs, key_index=kidx, tile_blocks=args.tile)
    t_plan = time.perf_counter() - t0
    t_batch = timed(batch.run, args.iters)
    res["batch"] = {"ms": round(t_batch * 1e3, 3), "msgs_per_s": round(n / t_batch), "gbps": round(n * size / t_batch / 1e9, 3),
                    "plan_ms": round(t_plan * 1e3, 3), "tiles": batch.ntiles, "tile_blocks": batch.tile_blocks}
    # the same messages described as one packed buffer: vectorised planning
    t0 = time.perf_counter()
    packed = ops.CtrBatch.packed(src, [size] * n, keys, ctrs, out=dst, key_index=kidx, tile_blocks=args.tile)
    t_plan_p = time.perf_counter() - t0
    t_packed = timed(packed.run, args.iters)
    res["batch_packed"] = {"ms": round(t_packed * 1e3, 3), "gbps": round(n * size / t_packed / 1e9, 3),
                           "plan_ms": round(t_plan_p * 1e3, 3)}
    if "eager" in res:
        res["batch_vs_eager"] = round(t_eager / t_batch, 1)
        res["batch_vs_graph"] = round(t_graph / t_batch, 1)
    ok = True
    for i in (0, n // 2, n - 1):
        ok = ok and outs[i].cpu().numpy().tobytes() == cpu_ref.ctr(keys[kidx[i]], ctrs[i], xs[i].cpu().numpy().tobytes())
    res["verified_sample"] = bool(ok)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
