#!/usr/bin/env python3
"""BASELINE config 4: AES-256-CBC over one root-resident stream, DP-sharded
across the node's GPUs with RCCL scatter/gather over xGMI.

One process per GPU (torchrun).  The root GPU produces the plaintext stream
chunk by chunk (synthetic random bytes, generated on the root so the host
link is not the bottleneck), scatters equal pieces (RCCL scatter = one-hop
fan-out over the root's 7 xGMI links), every rank CBC-encrypts its piece as
independent 4 KiB sectors (IV_s = iv0 + global sector index -- the parallel
CBC semantic), and the ciphertext is gathered back to
the root.  Default total: 32 GiB per GPU (256 GiB at 8 GPUs), streamed in
rounds of --chunk-mib per rank, so nothing close to 256 GiB is ever resident.

The rounds run through parallel.dist.ScatterGatherPipeline: the gather of
round r (root ingress) is issued asynchronously on its own communicator and
overlaps the scatter of round r+1 (root egress) -- xGMI links are full
duplex.  --no-overlap serialises both on one communicator (A/B).

--decrypt: exact single-stream CBC decryption instead -- every scattered
piece carries the 16-byte ciphertext block in front of it (the halo), so each
rank decrypts its piece independently and the gathered result equals the
serial decryption of the whole stream.

Every rank's piece is verified (checksums of what it received and produced
against what the root sent and gathered, plus an oracle sample of its
output) after the first and the last round; a failed rank fails the run.
Even at one GPU the job runs through a (1-rank) RCCL process group with the
duplex communicators, so the collective code path is what is measured.

    python benchmarks/cbc_scatter.py --gpus 8                # self-spawns 8 ranks
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/cbc_scatter.py --gpus 8
    python benchmarks/cbc_scatter.py --gib-per-gpu 4         # 1 GPU
"""
import argparse
import json
import os

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # before torch / HIP: dmabuf IPC only on this host driver (as bench.py)
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU); spawned here without a launcher")
    ap.add_argument("--timeout", type=float, default=3600.0, help="seconds before a self-spawned run is stopped")
    ap.add_argument("--gib-per-gpu", type=float, default=32.0)
    ap.add_argument("--chunk-mib", type=int, default=1024, help="per-rank bytes per scatter round")
    ap.add_argument("--sector", type=int, default=4096)
    ap.add_argument("--bits", type=int, default=256)
    ap.add_argument("--no-overlap", action="store_true", help="serial scatter -> encrypt -> gather rounds")
    ap.add_argument("--decrypt", action="store_true",
                    help="exact single-stream CBC decryption: every piece travels with its 16-byte halo")
    args = ap.parse_args()

    # the launch is decided before anything touches the GPU (parallel/launch.py)
    from our_tree_amd.parallel import launch

    launch.dispatch(args.gpus, os.path.abspath(__file__), sys.argv[1:], timeout_s=args.timeout)

    import torch

    from our_tree_amd.parallel import dist as pdist
    from our_tree_amd.parallel import jobs

    rank, world, local = pdist.init_from_env(force=True)
    assert world == args.gpus, (world, args.gpus)
    dev = torch.device("cuda", local)
    chunk = args.chunk_mib << 20
    total = int(args.gib_per_gpu * (1 << 30)) * world
    total -= total % (chunk * world)
    rounds = total // (chunk * world)
    res = jobs.cbc_scatter_job(rounds, chunk, bytes(range(args.bits // 8)), bytes(range(0xA0, 0xB0)),
                               sector=args.sector, decrypt=args.decrypt, overlap=not args.no_overlap, device=dev)
    if rank == 0:
        what = "decrypt, exact single stream (halos)" if args.decrypt else "sector-parallel encrypt"
        print(json.dumps({"metric": f"GB/s AES-{args.bits}-CBC ({what}) root scatter/gather",
                          "n_gpus": world, "total_bytes": res["total_bytes"], "rounds": rounds,
                          "chunk_per_rank": chunk, "overlap": res["overlap"], "seconds": round(res["seconds"], 3),
                          "value": round(res["gbps"], 3), "unit": "GB/s", "verified_sample": res["verified"],
                          "ranks": res["ranks"], "ranks_verified": res["ranks_verified"],
                          "backend": res["backend"], "collectives": res["collectives"],
                          "transport": res["transport"],
                          "xgmi_bytes_verified": res["xgmi_bytes_verified"],
                          "host_bytes_verified": res["host_bytes_verified"],
                          "xgmi_bytes_timed": res["xgmi_bytes_timed"],
                          "data": "synthetic random (root GPU fill)"}), flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()
    sys.exit(0 if res["verified"] else 1)


if __name__ == "__main__":
    main()
