#!/usr/bin/env python3
"""BASELINE config 5: AES-128-CTR over a host-resident stream, streamed through
every GPU with the native pinned pipeline (H2D(k+1) | kernel(k) | D2H(k-1) on
three HIP streams, csrc/hip/engine.cpp).

One process per GPU (torchrun); rank r owns the r-th contiguous share of the
logical stream and its counter offset.  A host box cannot hold 1 TiB, so each
rank re-streams a pinned host window of --window-gib (plaintext repeats, the
counter -- and therefore the keystream -- does not) until its share of
--total-gib has crossed PCIe both ways.  Default: 1 TiB over the node.

    python benchmarks/stream_ctr.py --gpus 8            # self-spawns 8 ranks
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/stream_ctr.py --gpus 8
    python benchmarks/stream_ctr.py --total-gib 32      # 1 GPU
"""
import argparse
import json
import os

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # before torch / HIP: dmabuf IPC only on this host driver (as bench.py)
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU); spawned here without a launcher")
    ap.add_argument("--timeout", type=float, default=3600.0, help="seconds before a self-spawned run is stopped")
    ap.add_argument("--total-gib", type=float, default=1024.0)
    ap.add_argument("--window-gib", type=float, default=4.0)
    ap.add_argument("--chunk-mib", type=int, default=64)
    args = ap.parse_args()

    # the launch is decided before anything touches the GPU (parallel/launch.py)
    from our_tree_amd.parallel import launch

    launch.dispatch(args.gpus, os.path.abspath(__file__), sys.argv[1:], timeout_s=args.timeout)

    import torch

    from our_tree_amd.models import cpu_ref
    from our_tree_amd.parallel import dist as pdist
    from our_tree_amd.parallel import stream as pstream

    rank, world, local = pdist.init_from_env()
    assert world == args.gpus, (world, args.gpus)
    share = int(args.total_gib * (1 << 30)) // world
    win = min(share, int(args.window_gib * (1 << 30)))
    win -= win % 16
    share -= share % win
    key, ctr0 = bytes(range(16)), bytes(range(0xF0, 0x100))
    hin = pstream.pinned_empty(win)
    hout = pstream.pinned_empty(win)
    rng = np.random.default_rng(rank)
    hin[:] = rng.integers(0, 256, win, dtype=np.uint8)
    base_blk = rank * (share // 16)
    with pstream.StreamEngine(local, chunk_bytes=args.chunk_mib << 20, depth=3) as eng:
        eng.run("ctr", hin, hout, key, ctr0, block_offset=base_blk)  # warmup + verification
        S = 1 << 16
        ok = hout[:S].tobytes() == cpu_ref.ctr(key, ctr0, hin[:S].tobytes(), base_blk)
        if world > 1:
            torch.distributed.barrier()
        t0 = time.perf_counter()
        h2d = d2h = 0.0
        npass = share // win
        for p in range(npass):
            st = eng.run("ctr", hin, hout, key, ctr0, block_offset=base_blk + p * (win // 16))
            h2d += st["h2d_gbps"] / npass
            d2h += st["d2h_gbps"] / npass
        el = pdist.allreduce_max(time.perf_counter() - t0)
        numa = eng.numa_node
    ok_all = pdist.allreduce_max(0.0 if ok else 1.0) == 0.0
    row = torch.tensor([float(rank), float(numa), h2d, d2h], dtype=torch.float64)
    rows = [row]
    if world > 1:
        dev = torch.device("cuda", local) if torch.distributed.get_backend() == "nccl" else "cpu"
        rows = [torch.empty(4, dtype=torch.float64, device=dev) for _ in range(world)]
        torch.distributed.all_gather(rows, row.to(dev))
    if rank == 0:
        tot = share * world
        print(json.dumps({"metric": "GB/s AES-128-CTR host-streamed (pinned H2D/D2H overlap)", "n_gpus": world,
                          "total_bytes": tot, "window_bytes": win, "chunk": args.chunk_mib << 20,
                          "seconds": round(el, 3), "value": round(tot / el / 1e9, 3), "unit": "GB/s",
                          "verified_sample": ok_all,
                          "per_rank": [{"rank": int(r[0]), "numa_node": int(r[1]), "h2d_gbps": round(float(r[2]), 2),
                                        "d2h_gbps": round(float(r[3]), 2)} for r in (x.cpu().tolist() for x in rows)],
                          "data": "synthetic random host window, re-streamed"}),
              flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()
    sys.exit(0 if ok_all else 1)


if __name__ == "__main__":
    main()
