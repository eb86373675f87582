#!/usr/bin/env python3
"""BASELINE config 4: AES-256-CBC over one root-resident stream, DP-sharded
across the node's GPUs with RCCL scatter/gather over xGMI.

One process per GPU (torchrun).  The root GPU produces the plaintext stream
chunk by chunk (synthetic random bytes, generated on the root so the host
link is not the bottleneck), scatters equal pieces (RCCL scatter = one-hop
fan-out over the root's 7 xGMI links), every rank CBC-encrypts its piece as
independent 4 KiB sectors (IV_s = iv0 + global sector index -- the parallel
CBC semantic), and the ciphertext is gathered back to
the root.  Default total: 32 GiB per GPU (256 GiB at 8 GPUs).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/cbc_scatter.py
    python benchmarks/cbc_scatter.py --gib-per-gpu 4        # 1 GPU
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from our_tree_amd import ops  # noqa: E402
from our_tree_amd.models import cpu_ref  # noqa: E402
from our_tree_amd.parallel import dist as pdist  # noqa: E402
from our_tree_amd.parallel import shard as sh  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib-per-gpu", type=float, default=32.0)
    ap.add_argument("--chunk-mib", type=int, default=1024, help="per-rank bytes per scatter round")
    ap.add_argument("--sector", type=int, default=4096)
    ap.add_argument("--bits", type=int, default=256)
    args = ap.parse_args()

    rank, world, local = pdist.init_from_env()
    dev = torch.device("cuda", local)
    chunk = args.chunk_mib << 20
    total = int(args.gib_per_gpu * (1 << 30)) * world
    total -= total % (chunk * world)
    key = bytes(range(args.bits // 8))
    iv0 = bytes(range(0xA0, 0xB0))
    seg = args.sector

    src = torch.empty(chunk * world, dtype=torch.uint8, device=dev) if rank == 0 else None
    recv = torch.empty(chunk, dtype=torch.uint8, device=dev)
    ct = torch.empty(chunk, dtype=torch.uint8, device=dev)
    gathered = torch.empty(chunk * world, dtype=torch.uint8, device=dev) if rank == 0 else None
    rounds = total // (chunk * world)

    def one_round(r, check=False):
        if rank == 0:
            ops.fill_random_(src, seed=r)
        if world > 1:
            dist.scatter(recv, list(src.chunk(world)) if rank == 0 else None, src=0)
        else:
            recv.copy_(src)
        gofs = (r * world + rank) * chunk
        ivr = sh.ctr_add(iv0, gofs // seg)
        ops.cbc_encrypt_segments(recv, key, ivr, seg, out=ct)
        if world > 1:
            dist.gather(ct, list(gathered.chunk(world)) if rank == 0 else None, dst=0)
        else:
            gathered.copy_(ct)
        if check and rank == 0:
            torch.cuda.synchronize()
            n = 4 * seg
            pt = src[:n].cpu().numpy().tobytes()
            exp = cpu_ref.cbc_segments(key, sh.ctr_add(iv0, (r * world) * chunk // seg), pt, seg)
            return gathered[:n].cpu().numpy().tobytes() == exp
        return True

    ok = one_round(0, check=True)  # warmup + verification (outside timing)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for r in range(rounds):
        one_round(r)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = pdist.allreduce_max(time.perf_counter() - t0)
    if rank == 0:
        print(json.dumps({"metric": f"GB/s AES-{args.bits}-CBC (sector-parallel) root scatter/gather", "n_gpus": world,
                          "total_bytes": total, "rounds": rounds, "chunk_per_rank": chunk, "seconds": round(el, 3),
                          "value": round(total / el / 1e9, 3), "unit": "GB/s", "verified_sample": bool(ok),
                          "data": "synthetic random (root GPU fill)"}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
