#!/usr/bin/env python3
"""Headline benchmark: whole-node AES-128-CTR throughput (GB/s) on MI355X.

Metric and config come from BASELINE.json ("GB/s AES-128-CTR (whole node) at
1/2/4/8 MI355X; cycles/byte per CU"; config "AES-128-CTR 64 GiB ... one
MI355X").  One process per GPU (torchrun), each rank owns a 64 GiB shard of one
logical plaintext stream in HBM (synthetic random bytes, random key) and
encrypts it in place with the counter offset of its shard (rank * shard_blocks)
-- weak scaling, 64 GiB per GPU.  A step = one full pass over every shard.
Timing: W untimed warmup steps, barrier + synchronize, K timed steps,
synchronize + barrier, MAX over ranks.  Correctness is checked on a sample of
every shard against the CPU oracle before timing.

Multi-GPU: ``python bench.py --gpus N`` without a launcher spawns N fresh
worker processes itself (parallel/launch.py) before anything touches the GPU;
under torchrun WORLD_SIZE must equal --gpus.  Fewer visible GPUs than --gpus
is an error (exit 2) -- a multi-GPU request is never measured on fewer GPUs.

Communication: the resident CTR step needs none (every rank owns its shard),
so an extra, separately timed pass runs BASELINE config 4 in miniature -- an
AES-256-CBC stream on the root GPU dealt to all ranks by RCCL scatter over
xGMI, sector-encrypted, gathered back.  Every rank's received and produced
piece is checksummed against what the root sent and gathered, and a sample
of every rank's output is checked against the C oracle (``rccl_ranks_verified``);
the xGMI bytes reported are those of the verified pieces.  A second extra
streams a few GiB per rank from pinned, NUMA-placed host memory through the
3-stream H2D | kernel | D2H pipeline (BASELINE config 5 in miniature) and
reports every rank's NUMA node and per-direction PCIe rate.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--gib 64]
        torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_GBPS = 0.519  # BASELINE.md headline CTR: AES-NI CTR-256, 1000 MiB, 8 threads (frankchn)
BASELINE_GPU_GBPS = 2.41  # BASELINE.md repo headline: CUDA "AES ECB" 1000 MiB (baryon)
AES128_EQUIV = 14 / 10  # AES-256 -> AES-128 round ratio (BASELINE.md caveat 5: derived, not published)


def baseline_ratios(value: float) -> dict:
    """The headline's ratios to BASELINE.md, each labelled.  The reference
    publishes AES-256 numbers only, so ``vs_baseline`` divides AES-128 bytes by
    the AES-256 CPU headline; ``vs_baseline_aes128_equiv`` scales that
    baseline by the round ratio (derived, not published); the like-for-like
    AES-256 ratio is the ``aes256_vs_cpu_aesni_ctr256`` extra."""
    return {
        "vs_baseline": round(value / BASELINE_GBPS, 2),
        "vs_baseline_what": "AES-128-CTR GB/s / 0.519 GB/s AES-NI CTR-256 1000 MiB 8 threads "
                            "(aes-modes/results.frankchn.aesni:32; no AES-128 number is published)",
        "vs_baseline_aes128_equiv": round(value / (BASELINE_GBPS * AES128_EQUIV), 2),
    }


def stream_pass(args, key, counter, rank, world, local, block0):
    """Host-streamed AES-128-CTR through the native pinned pipeline
    (H2D(k+1) | kernel(k) | D2H(k-1) on three HIP streams, staging ring on the
    GPU's NUMA node): each rank streams its own pinned host window
    ``--stream-passes`` times (counter advancing, so no keystream repeats),
    timed between barriers, MAX over ranks.  Returns the bench extras."""
    import numpy as np

    from our_tree_amd.models import cpu_ref
    from our_tree_amd.parallel import dist as pdist
    from our_tree_amd.parallel import stream as pstream

    win = int(args.stream_gib * (1 << 30))
    win -= win % 16
    hin = pstream.pinned_empty(win)
    hout = pstream.pinned_empty(win)
    rng = np.random.default_rng(7 + rank)
    hin[:] = rng.integers(0, 256, win, dtype=np.uint8)
    # stream blocks after the resident shards, so no counter is reused
    base = world * (int(args.gib * (1 << 30)) // 16) + rank * args.stream_passes * (win // 16)
    with pstream.StreamEngine(local, chunk_bytes=64 << 20, depth=3) as eng:
        eng.run("ctr", hin, hout, key, counter, block_offset=base)  # warmup + verification
        S = 1 << 16
        ok = (hout[:S].tobytes() == cpu_ref.ctr(key, counter, hin[:S].tobytes(), base)
              and hout[win - S:].tobytes() == cpu_ref.ctr(key, counter, hin[win - S:].tobytes(),
                                                         base + (win - S) // 16))
        if torch.distributed.is_initialized():
            torch.distributed.barrier()
        t0 = time.perf_counter()
        h2d = d2h = 0.0
        for p in range(args.stream_passes):
            st = eng.run("ctr", hin, hout, key, counter, block_offset=base + p * (win // 16))
            h2d += st["h2d_gbps"] / args.stream_passes
            d2h += st["d2h_gbps"] / args.stream_passes
        mine = time.perf_counter() - t0
        numa = eng.numa_node
    el = pdist.allreduce_max(mine)
    ok_all = pdist.allreduce_max(0.0 if ok else 1.0) == 0.0
    row = [float(rank), float(numa), h2d, d2h, win * args.stream_passes / mine / 1e9]
    rows = [row]
    if torch.distributed.is_initialized():
        dev = torch.device("cuda", local) if torch.distributed.get_backend() == "nccl" else "cpu"
        t = torch.tensor(row, dtype=torch.float64, device=dev)
        outs = [torch.empty_like(t) for _ in range(world)]
        torch.distributed.all_gather(outs, t)
        rows = [o.cpu().tolist() for o in outs]
    del hin, hout
    return {
        "stream_ctr_gbps_whole_node": round(win * args.stream_passes * world / el / 1e9, 3),
        "stream_ctr_bytes_per_rank": win * args.stream_passes,
        "stream_ctr_verified": ok_all,
        "stream_ctr_per_rank": [{"rank": int(r[0]), "numa_node": int(r[1]), "h2d_gbps": round(r[2], 2),
                                 "d2h_gbps": round(r[3], 2), "gbps": round(r[4], 2)} for r in rows],
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--gib", type=float, default=64.0, help="per-GPU shard size in GiB")
    ap.add_argument("--impl", default=os.environ.get("OTC_BENCH_IMPL", "auto"))
    ap.add_argument("--no-aes256", action="store_true")
    ap.add_argument("--no-bitslice", "--no-other-impl", dest="no_other", action="store_true",
                    help="skip timing the other AES-128 CTR kernel (T-table vs bitsliced) on the same shard")
    ap.add_argument("--no-clock", action="store_true")
    ap.add_argument("--no-scatter", action="store_true", help="skip the RCCL scatter/gather AES-256-CBC pass")
    ap.add_argument("--scatter-mib", type=int, default=512, help="per-rank bytes per scatter round (MiB)")
    ap.add_argument("--scatter-rounds", type=int, default=4)
    ap.add_argument("--no-stream", action="store_true", help="skip the host-streamed CTR pass")
    ap.add_argument("--stream-gib", type=float, default=2.0, help="pinned host window per rank (GiB)")
    ap.add_argument("--stream-passes", type=int, default=3)
    ap.add_argument("--timeout", type=float, default=1800.0,
                    help="seconds before a self-spawned multi-GPU run is stopped (all ranks)")
    args = ap.parse_args()

    # decide the launch before any HIP call (spawned ranks re-enter here with
    # RANK/WORLD_SIZE set); exits on error or when the spawned run finished
    from our_tree_amd.parallel import launch

    launch.dispatch(args.gpus, os.path.abspath(__file__), sys.argv[1:], timeout_s=args.timeout)

    # stdout carries exactly one JSON line (rank 0): everything else written
    # to fd 1 from here on -- RCCL's version banner, library chatter -- goes
    # to stderr, and the result is written to the saved descriptor
    sys.stdout.flush()
    result_fd = os.dup(1)
    os.dup2(2, 1)

    def emit(obj):
        os.write(result_fd, (json.dumps(obj) + "\n").encode())

    from our_tree_amd import ops
    from our_tree_amd.models import cpu_ref
    from our_tree_amd.parallel import dist as pdist
    from our_tree_amd.utils import device as dinfo

    # The clock probe's stream is created before RCCL creates its streams: a
    # later one shared a hardware queue with the compute stream (4 per process
    # here), so the probe ran after the steps and read the idle clock (2.4 GHz
    # instead of the ~2.0 held under load).
    gpu = pdist.local_gpu()
    torch.cuda.set_device(gpu)
    probe_stream = torch.cuda.Stream(device=gpu, priority=-1)

    # a process group even at N=1 (a 1-rank RCCL group) so the scatter pass
    # always runs the collective code path
    rank, world, local = pdist.init_from_env(force=not args.no_scatter)
    assert world == args.gpus, (world, args.gpus)  # launch.dispatch guarantees it
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    nbytes = int(args.gib * (1 << 30))
    nbytes -= nbytes % 16
    gen = torch.Generator().manual_seed(1337)
    key = bytes(torch.randint(0, 256, (16,), generator=gen, dtype=torch.uint8).tolist())
    key256 = bytes(torch.randint(0, 256, (32,), generator=gen, dtype=torch.uint8).tolist())
    counter = bytes(torch.randint(0, 256, (16,), generator=gen, dtype=torch.uint8).tolist())
    shard_blocks = nbytes // 16
    my_block0 = rank * shard_blocks

    buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    ops.fill_random_(buf, seed=1000 + rank)

    # ---- correctness on a sample (outside the timed region) ----------------
    S = 1 << 16
    head = buf[:S].cpu().numpy().tobytes()
    tail_off = nbytes - S
    tail = buf[tail_off:].cpu().numpy().tobytes()
    ops.ctr(buf, key, counter, out=buf, block_offset=my_block0, impl=args.impl)
    torch.cuda.synchronize()
    ok = (buf[:S].cpu().numpy().tobytes() == cpu_ref.ctr(key, counter, head, my_block0)
          and buf[tail_off:].cpu().numpy().tobytes()
          == cpu_ref.ctr(key, counter, tail, my_block0 + tail_off // 16))
    ok_all = pdist.allreduce_max(0.0 if ok else 1.0) == 0.0
    if not ok_all:
        if rank == 0:
            emit({"error": "verification failed"})
        sys.exit(1)

    def step(k=key, impl=args.impl):
        ops.ctr(buf, k, counter, out=buf, block_offset=my_block0, impl=impl)

    def timed(nsteps, k, impl=args.impl):
        for _ in range(args.warmup):
            step(k, impl)
        torch.cuda.synchronize()
        if torch.distributed.is_initialized():
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(nsteps):
            step(k, impl)
        torch.cuda.synchronize()
        if torch.distributed.is_initialized():
            torch.distributed.barrier()
        el = time.perf_counter() - t0
        return pdist.allreduce_max(el)

    resolved = ops.pick_impl(args.impl, 128, "ctr", nbytes)  # the kernel the headline runs
    elapsed = timed(args.steps, key)
    ms_per_step = elapsed / args.steps * 1e3
    total_bytes = nbytes * world * args.steps
    value = total_bytes / elapsed / 1e9

    info = dinfo.info(local)
    cpb = (ms_per_step * 1e-3) * info["clock_hz"] * info["cus"] / nbytes

    # Clock the chip holds under this load (untimed extra steps with the
    # one-wave probe beside them): cycles/byte/CU at the nominal clock
    # overstates the cycle count when the chip lowers its clock.
    clk_ghz = None
    if not args.no_clock:
        n_clk = max(3, int(0.3 / max(ms_per_step * 1e-3, 1e-6)) + 1)
        window = 0.6 * n_clk * ms_per_step * 1e-3
        probe = ops.clock_probe(0.2 * n_clk * ms_per_step * 1e-3, window, device=dev, stream=probe_stream)
        for _ in range(n_clk):
            step()
        torch.cuda.synchronize()
        clk_ghz = ops.clock_ghz(probe)
    cpb_eff = (ms_per_step * 1e-3) * clk_ghz * 1e9 * info["cus"] / nbytes if clk_ghz else None

    extra = {}
    if not args.no_other:
        # the other AES-128 CTR kernel on the same shard, same protocol: the
        # headline's "auto" runs the bitsliced VALU kernel at this size (BASELINE
        # config 3 names it), the LDS T-table kernel is timed beside it
        other = "ttable" if resolved == "bitslice" else "bitslice"
        o_steps = max(1, min(args.steps, 5))
        el_o = timed(o_steps, key, impl=other)
        extra[("ttable" if other == "ttable" else "bitsliced") + "_ctr_gbps_whole_node"] = round(
            nbytes * world * o_steps / el_o / 1e9, 3)
    if not args.no_aes256:
        k256_steps = max(1, min(args.steps, 5))
        el256 = timed(k256_steps, key256)
        extra["aes256_ctr_gbps_whole_node"] = round(nbytes * world * k256_steps / el256 / 1e9, 3)
        extra["aes256_vs_cpu_aesni_ctr256"] = round(extra["aes256_ctr_gbps_whole_node"] / BASELINE_GBPS, 1)

    if not args.no_stream:
        extra.update(stream_pass(args, key, counter, rank, world, local, my_block0))
        if not extra["stream_ctr_verified"]:
            if rank == 0:
                emit({"error": "host-streamed CTR verification failed", **extra})
            sys.exit(1)

    if not args.no_scatter:
        from our_tree_amd.parallel import jobs

        del buf  # the scatter pass needs its own buffers (4 x world x chunk on the root)
        torch.cuda.empty_cache()
        sc = jobs.cbc_scatter_job(args.scatter_rounds, args.scatter_mib << 20, key256,
                                  bytes(range(0xA0, 0xB0)), sector=4096, device=dev)
        extra["rccl_cbc256_scatter_gbps"] = round(sc["gbps"], 3)
        extra["rccl_ranks"] = sc["ranks"]
        extra["rccl_ranks_verified"] = sc["ranks_verified"]
        extra["rccl_backend"] = sc["backend"]
        extra["rccl_xgmi_bytes_verified"] = sc["xgmi_bytes_verified"]
        extra["rccl_xgmi_bytes_timed"] = sc["xgmi_bytes_timed"]
        extra["rccl_scatter_bytes"] = sc["total_bytes"]
        extra["rccl_scatter_verified"] = sc["verified"]
        if not sc["verified"]:
            if rank == 0:
                emit({"error": "RCCL scatter/gather verification failed", "per_rank_ok": sc["per_rank_ok"], **extra})
            sys.exit(1)

    if rank == 0:
        line = {
            "metric": "GB/s AES-128-CTR (whole node)",
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            **baseline_ratios(value),
            "dtype": "uint8",  # cipher engine: byte data, no floating-point compute
            "data": "synthetic random plaintext (splitmix64), random 128-bit key and counter",
            "config": {
                "model": "AES-128-CTR",
                "global_batch": nbytes * world,
                "seq_len": nbytes,
                "parallelism": f"dp{world}",
                "per_gpu_bytes": nbytes,
                "in_place": True,
                "impl": args.impl,
                "impl_resolved": resolved,
            },
            "cycles_per_byte_per_cu": round(cpb, 4),
            "cycles_per_byte_per_cu_at_held_clock": round(cpb_eff, 4) if cpb_eff else None,
            "held_clock_ghz": round(clk_ghz, 3) if clk_ghz else None,
            "per_gpu_gbps": round(value / world, 3),
            "baseline": {"value_gbps": BASELINE_GBPS, "what": "AES-NI CTR-256 1000MiB 8thr (BASELINE.md)",
                         "gpu_headline_gbps": BASELINE_GPU_GBPS},
            "verified_sample": True,
            **extra,
        }
        emit(line)
    if torch.distributed.is_initialized():
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
