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

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/cbc_scatter.py
    python benchmarks/cbc_scatter.py --gib-per-gpu 4        # 1 GPU
"""
import argparse
import json
import os
import sys
import time

import torch

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
    ap.add_argument("--no-overlap", action="store_true", help="serial scatter -> encrypt -> gather rounds")
    ap.add_argument("--decrypt", action="store_true",
                    help="exact single-stream CBC decryption: every piece travels with its 16-byte halo")
    args = ap.parse_args()

    rank, world, local = pdist.init_from_env()
    dev = torch.device("cuda", local)
    chunk = args.chunk_mib << 20
    total = int(args.gib_per_gpu * (1 << 30)) * world
    total -= total % (chunk * world)
    rounds = total // (chunk * world)
    key = bytes(range(args.bits // 8))
    iv0 = bytes(range(0xA0, 0xB0))
    seg = args.sector
    # decrypt: a piece is [16-byte halo | chunk of ciphertext]; the halo is the
    # ciphertext block in front of the chunk in the single stream (the IV for
    # the very first one), so every rank decrypts exactly
    H = 16 if args.decrypt else 0
    piece_bytes = chunk + H
    pipe = pdist.ScatterGatherPipeline(piece_bytes, root=0, device=dev, overlap=not args.no_overlap)
    carry = torch.tensor(list(iv0), dtype=torch.uint8, device=dev)  # last block of the previous round (root)

    def produce(send, r):
        if not args.decrypt:
            ops.fill_random_(send, seed=r)
            return
        v = send.view(world, piece_bytes)
        for g in range(world):  # synthetic ciphertext, piece by piece (rows are strided)
            ops.fill_random_(v[g, H:], seed=r * world + g)
        v[0, :H].copy_(carry)
        v[1:, :H].copy_(v[:-1, -H:])
        carry.copy_(v[-1, -H:])

    def work(piece, out, r):
        if not args.decrypt:
            gofs = (r * world + rank) * chunk
            ops.cbc_encrypt_segments(piece, key, sh.ctr_add(iv0, gofs // seg), seg, out=out)
            return
        # IV 0, then XOR the halo into the first block: no host round trip
        ops.cbc_decrypt(piece[H:], key, bytes(16), out=out[H:])
        out[H:2 * H].bitwise_xor_(piece[:H])

    verdict = {}

    def verify(gathered, r):
        """first sectors of rank 0's and the last rank's pieces vs the oracle
        (warmup round only, outside the timed region)"""
        torch.cuda.synchronize()
        n = 4 * seg
        ok = True
        send = pipe.send[r % len(pipe.send)]
        for g in (0, world - 1):
            a = g * piece_bytes
            src = send[a + H:a + H + n].cpu().numpy().tobytes()
            if args.decrypt:
                exp = cpu_ref.cbc(key, send[a:a + H].cpu().numpy().tobytes(), src, decrypt=True)
            else:
                exp = cpu_ref.cbc_segments(key, sh.ctr_add(iv0, (r * world + g) * chunk // seg), src, seg)
            ok = ok and gathered[a + H:a + H + n].cpu().numpy().tobytes() == exp
        if args.decrypt and world > 1:  # halo of rank 1 = last ciphertext block of rank 0
            ok = ok and torch.equal(send[piece_bytes:piece_bytes + H], send[piece_bytes - H:piece_bytes])
        verdict["ok"] = ok

    pipe.run(1, produce, work, verify)  # warmup + verification
    torch.cuda.synchronize()
    if torch.distributed.is_initialized():
        torch.distributed.barrier()
    t0 = time.perf_counter()
    pipe.run(rounds, produce, work)
    torch.cuda.synchronize()
    if torch.distributed.is_initialized():
        torch.distributed.barrier()
    el = pdist.allreduce_max(time.perf_counter() - t0)
    if rank == 0:
        what = "decrypt, exact single stream (halos)" if args.decrypt else "sector-parallel encrypt"
        print(json.dumps({"metric": f"GB/s AES-{args.bits}-CBC ({what}) root scatter/gather",
                          "n_gpus": world, "total_bytes": total, "rounds": rounds, "chunk_per_rank": chunk,
                          "overlap": pipe.overlap, "seconds": round(el, 3), "value": round(total / el / 1e9, 3),
                          "unit": "GB/s", "verified_sample": bool(verdict.get("ok")),
                          "data": "synthetic random (root GPU fill)"}), flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
