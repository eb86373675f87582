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

Per rank (``per_rank``): its own GB/s over the same steps, the clock it held,
its verification, and -- the chip runs against its package power limit, so
throughput follows energy per byte -- the socket energy over exactly the timed
steps (amdsmi energy counter), average power, J/GB and the fraction of the
window the PPT limit was active.  Whole node: ``joules_per_gb``,
``avg_socket_w_per_gpu``, ``ppt_residency_max``.

Multi-GPU: ``python bench.py --gpus N`` without a launcher spawns N fresh
worker processes itself (parallel/launch.py) before anything touches the GPU;
under torchrun WORLD_SIZE must equal --gpus.  Fewer visible GPUs than --gpus
is an error (exit 2) -- a multi-GPU request is never measured on fewer GPUs.
Before any large allocation a bounded preflight moves 16 MiB through a scatter
and an all_gather and checks every byte (parallel/preflight.py): a broken
peer transport ends the run with one error JSON line after --preflight-timeout
seconds instead of hanging.

Communication: the resident CTR step needs none (every rank owns its shard),
so an extra, separately timed pass runs BASELINE config 4 in miniature -- an
AES-256-CBC stream on the root GPU dealt to all ranks by RCCL scatter over
xGMI, sector-encrypted, gathered back.  Every rank's received and produced
piece is checksummed against what the root sent and gathered, and a sample
of every rank's output is checked against the C oracle (``rccl_ranks_verified``);
the xGMI bytes reported are those of the verified pieces.  A second extra
streams a few GiB per rank from pinned, NUMA-placed host memory through the
3-stream H2D | kernel | D2H pipeline (BASELINE config 5 in miniature) and
reports every rank's NUMA node and per-direction PCIe rate.  A third reruns
the reference's own GPU measurement (AES-256 ECB, 1000 MiB, allocation and
pageable copies inside the timer, main_ecb_e.cu:37-44) beside the pinned and
kernel-only figures for the same buffer (utils/refmethod.py).

``--device cpu`` rehearses the whole flow (launch, preflight, per-rank
gather, JSON) on the host with gloo and the C oracle, tiny shards.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--gib 64]
        torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import os

# Before torch / HIP load, for every way this script is started (self-spawned
# ranks, torchrun, plain python): this host driver supports dmabuf IPC only,
# and RCCL's peer transport fails (hipIpcGetMemHandle: invalid argument)
# without it.  setdefault: an explicit value from the caller wins.
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import argparse  # noqa: E402
import json  # noqa: E402
import sys  # noqa: E402
import time  # noqa: E402

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_GBPS = 0.519  # BASELINE.md headline CTR: AES-NI CTR-256, 1000 MiB, 8 threads (frankchn)
BASELINE_GPU_GBPS = 2.41  # BASELINE.md repo headline: CUDA "AES ECB" 1000 MiB (baryon)
AES128_EQUIV = 14 / 10  # AES-256 -> AES-128 round ratio (BASELINE.md caveat 5: derived, not published)
RANK_KEYS = ("gbps", "held_clock_ghz", "verified", "joules", "energy_gb", "avg_socket_w", "joules_per_gb",
             "ppt_residency", "gfxclk_mhz_mean", "xgmi_read_kb", "xgmi_write_kb")


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


def per_rank_table(rows: list[list[float]]) -> list[dict]:
    """Rows of floats in RANK_KEYS order (nan = not measured) -> one dict per
    rank, ``verified`` as a bool, unmeasured values as None."""
    out = []
    for r, row in enumerate(rows):
        d = {"rank": r}
        for k, v in zip(RANK_KEYS, row):
            if k == "verified":
                d[k] = bool(v == 1.0)
            elif v != v:  # nan
                d[k] = None
            elif k.startswith("xgmi"):
                d[k] = int(v)
            else:
                d[k] = round(v, 4 if k in ("joules_per_gb", "ppt_residency", "held_clock_ghz") else 3)
        out.append(d)
    return out


def node_energy(table: list[dict]) -> dict:
    """Whole-node energy keys from the per-rank table: J/GB = all ranks'
    socket energy over all the bytes their energy windows processed (None
    unless every rank read its counters)."""
    js = [d["joules"] for d in table if d["joules"] is not None]
    gb = [d["energy_gb"] for d in table if d["energy_gb"] is not None]
    ws = [d["avg_socket_w"] for d in table if d["avg_socket_w"] is not None]
    pp = [d["ppt_residency"] for d in table if d["ppt_residency"] is not None]
    full = len(js) == len(gb) == len(table)
    return {
        "joules_per_gb": round(sum(js) / sum(gb), 4) if full and js and sum(gb) > 0 else None,
        "avg_socket_w_per_gpu": round(sum(ws) / len(ws), 1) if ws else None,
        "ppt_residency_max": round(max(pp), 4) if pp else None,
        "energy_ranks": len(js),
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
    rows = pdist.gather_floats([float(rank), float(numa), h2d, d2h, win * args.stream_passes / mine / 1e9])
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
    ap.add_argument("--device", choices=("gpu", "cpu"), default="gpu",
                    help="cpu: rehearse the flow on the host (gloo, C oracle, tiny shards)")
    ap.add_argument("--no-aes256", action="store_true")
    ap.add_argument("--no-bitslice", "--no-other-impl", dest="no_other", action="store_true",
                    help="skip timing the other AES-128 CTR kernel (T-table vs bitsliced) on the same shard")
    ap.add_argument("--no-clock", action="store_true")
    ap.add_argument("--no-power", action="store_true", help="skip the amdsmi energy / power / PPT counters")
    ap.add_argument("--energy-min-s", type=float, default=2.0,
                    help="shortest energy window: untimed identical steps extend it after the timed ones")
    ap.add_argument("--no-scatter", action="store_true", help="skip the RCCL scatter/gather AES-256-CBC pass")
    ap.add_argument("--scatter-mib", type=int, default=512, help="per-rank bytes per scatter round (MiB)")
    ap.add_argument("--scatter-rounds", type=int, default=4)
    ap.add_argument("--no-stream", action="store_true", help="skip the host-streamed CTR pass")
    ap.add_argument("--stream-gib", type=float, default=2.0, help="pinned host window per rank (GiB)")
    ap.add_argument("--stream-passes", type=int, default=3)
    ap.add_argument("--no-refmethod", action="store_true",
                    help="skip the reference-methodology AES-256 ECB 1000 MiB rows")
    ap.add_argument("--timeout", type=float, default=1800.0,
                    help="seconds before a self-spawned multi-GPU run is stopped (all ranks)")
    ap.add_argument("--preflight-timeout", type=float, default=120.0)
    ap.add_argument("--preflight-fault-rank", type=int, default=None, help=argparse.SUPPRESS)  # test hook
    ap.add_argument("--preflight-hang-rank", type=int, default=None, help=argparse.SUPPRESS)  # test hook
    args = ap.parse_args()
    cpu = args.device == "cpu"
    if cpu:
        os.environ.setdefault("OTC_DIST_BACKEND", "gloo")
        os.environ.setdefault("OTC_SHARE_GPUS", "1")  # ranks are host processes: no GPU count applies
        args.no_clock = args.no_power = args.no_stream = args.no_refmethod = True

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

    from our_tree_amd.models import cpu_ref
    from our_tree_amd.parallel import dist as pdist
    from our_tree_amd.parallel import preflight

    probe_stream = None
    if not cpu:
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

    def on_timeout(r, t):
        msg = {"error": f"preflight: scatter/all_gather did not finish within {t:.0f} s "
                        "(peer transport / IPC failure?)", "rank": r}
        if r == 0:
            emit(msg)
        print(json.dumps(msg), file=sys.stderr, flush=True)
        os._exit(3)

    pre = preflight.run(timeout_s=args.preflight_timeout, on_timeout=on_timeout,
                        fault_rank=args.preflight_fault_rank, hang_rank=args.preflight_hang_rank)
    if not pre["ok"]:
        if rank == 0:
            emit({"error": "preflight verification failed", "preflight": pre})
        sys.exit(1)

    dev = torch.device("cpu") if cpu else torch.device("cuda", local)
    if not cpu:
        torch.cuda.set_device(dev)

    nbytes = int(args.gib * (1 << 30))
    nbytes -= nbytes % 16
    gen = torch.Generator().manual_seed(1337)
    key = bytes(torch.randint(0, 256, (16,), generator=gen, dtype=torch.uint8).tolist())
    key256 = bytes(torch.randint(0, 256, (32,), generator=gen, dtype=torch.uint8).tolist())
    counter = bytes(torch.randint(0, 256, (16,), generator=gen, dtype=torch.uint8).tolist())
    shard_blocks = nbytes // 16
    my_block0 = rank * shard_blocks

    def sync():
        if not cpu:
            torch.cuda.synchronize()

    buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    if cpu:
        buf.copy_(torch.randint(0, 256, (nbytes,), generator=torch.Generator().manual_seed(1000 + rank),
                                dtype=torch.uint8))
        resolved = "cpu-oracle"
    else:
        from our_tree_amd import ops

        ops.fill_random_(buf, seed=1000 + rank)
        resolved = ops.pick_impl(args.impl, 128, "ctr", nbytes)  # the kernel the headline runs

    def step(k=key, impl=args.impl):
        if cpu:
            pdist._ctr_local(buf, k, counter, my_block0)
        else:
            ops.ctr(buf, k, counter, out=buf, block_offset=my_block0, impl=impl)

    # ---- correctness on a sample (outside the timed region) ----------------
    S = min(1 << 16, nbytes // 2 - (nbytes // 2) % 16)

    def verify_once(k, impl=args.impl) -> bool:
        """one untimed step on the live (in-place) buffer, head and tail
        samples checked against the oracle -- run before each timed config"""
        head = buf[:S].cpu().numpy().tobytes()
        tail = buf[nbytes - S:].cpu().numpy().tobytes()
        step(k, impl)
        sync()
        return (buf[:S].cpu().numpy().tobytes() == cpu_ref.ctr(k, counter, head, my_block0)
                and buf[nbytes - S:].cpu().numpy().tobytes()
                == cpu_ref.ctr(k, counter, tail, my_block0 + (nbytes - S) // 16))

    ok = verify_once(key)
    ok_all = pdist.allreduce_max(0.0 if ok else 1.0) == 0.0
    if not ok_all:
        if rank == 0:
            emit({"error": "verification failed"})
        sys.exit(1)

    meter = None
    if not args.no_power:
        from our_tree_amd.utils.power import PowerMeter

        meter = PowerMeter(local)

    def timed(nsteps, k, impl=args.impl, measure=False, fn=None):
        """returns (MAX over ranks of the barrier-to-barrier time, this rank's
        own time to its last synchronize, power stats of this rank or None).
        With ``measure`` the energy window opens with the timed steps and,
        if they took less than --energy-min-s, stays open over identical
        untimed steps after the clock has stopped: the socket energy counter
        updates about every millisecond, so a short window reads ~0 J.
        ``fn(k, impl)``: the op timed (default: the headline's CTR step)."""
        fn = fn or step
        for _ in range(args.warmup):
            fn(k, impl)
        sync()
        if torch.distributed.is_initialized():
            torch.distributed.barrier()
        sync()
        if measure and meter is not None:
            meter.start()
        t0 = time.perf_counter()
        for _ in range(nsteps):
            fn(k, impl)
        sync()
        mine = time.perf_counter() - t0
        if torch.distributed.is_initialized():
            torch.distributed.barrier()
        el = time.perf_counter() - t0
        pw = None
        if measure and meter is not None:
            done = nsteps
            while time.perf_counter() - t0 < args.energy_min_s:
                fn(k, impl)
                done += 1
            sync()
            pw = meter.stop(nbytes * done)
            if pw.get("available"):
                pw["energy_steps"] = done
        return pdist.allreduce_max(el), mine, pw

    elapsed, mine, pw = timed(args.steps, key, measure=True)
    ms_per_step = elapsed / args.steps * 1e3
    total_bytes = nbytes * world * args.steps
    value = total_bytes / elapsed / 1e9

    clk_ghz = None
    cus, clock_hz = 256, 2.4e9
    if not cpu:
        from our_tree_amd.utils import device as dinfo

        info = dinfo.info(local)
        cus, clock_hz = info["cus"], info["clock_hz"]
        # Clock the chip holds under this load (untimed extra steps with the
        # one-wave probe beside them): cycles/byte/CU at the nominal clock
        # overstates the cycle count when the chip lowers its clock.
        if not args.no_clock:
            n_clk = max(3, int(0.3 / max(ms_per_step * 1e-3, 1e-6)) + 1)
            window = 0.6 * n_clk * ms_per_step * 1e-3
            probe = ops.clock_probe(0.2 * n_clk * ms_per_step * 1e-3, window, device=dev, stream=probe_stream)
            for _ in range(n_clk):
                step()
            torch.cuda.synchronize()
            clk_ghz = ops.clock_ghz(probe)
    cpb = (ms_per_step * 1e-3) * clock_hz * cus / nbytes
    cpb_eff = (ms_per_step * 1e-3) * clk_ghz * 1e9 * cus / nbytes if clk_ghz else None

    nan = float("nan")
    pwv = pw if pw and pw.get("available") else {}
    row = [nbytes * args.steps / mine / 1e9, clk_ghz if clk_ghz else nan, 1.0 if ok else 0.0]
    energy_gb = nbytes * pwv["energy_steps"] / 1e9 if pwv.get("energy_steps") else None
    row += [float(pwv["joules"]) if pwv.get("joules") is not None else nan, energy_gb if energy_gb else nan]
    row += [float(pwv[k]) if pwv.get(k) is not None else nan
            for k in ("avg_socket_w", "joules_per_gb", "ppt_residency", "gfxclk_mhz_mean", "xgmi_read_kb",
                      "xgmi_write_kb")]
    table = per_rank_table(pdist.gather_floats(row))
    energy = node_energy(table)
    # cycles/byte/CU at the clock amd-smi saw over each rank's energy window
    # (all 8 XCDs sampled every 50 ms) and that rank's own rate, the largest
    # over ranks: steadier than the one-wave probe's (r4/r5 records:
    # 0.2690-0.2717 where the probe read 0.269-0.2808)
    cpbs = [d["gfxclk_mhz_mean"] * 1e6 * cus / (d["gbps"] * 1e9) for d in table
            if d.get("gfxclk_mhz_mean") and d.get("gbps")]
    cpb_mean = max(cpbs) if cpbs and not cpu else None
    if pwv:
        energy["energy_window_s"] = pwv.get("window_s")  # rank 0's: timed steps + untimed extension
    if meter is not None and not pwv:
        energy["energy_unavailable"] = pw.get("reason") if pw else "no window"

    extra = {}
    if not args.no_other and not cpu:
        # the other AES-128 CTR kernel on the same shard, same protocol: the
        # headline's "auto" runs the bitsliced VALU kernel at this size (the
        # one BASELINE config 3 names); the LDS T-table is timed beside it
        for other in ("bitslice", "ttable"):
            if other == resolved:
                continue
            name = "ttable" if other == "ttable" else "bitsliced"
            v_ok = pdist.allreduce_max(0.0 if verify_once(key, other) else 1.0) == 0.0
            o_steps = max(1, min(args.steps, 5))
            el_o, _, _ = timed(o_steps, key, impl=other)
            extra[name + "_ctr_gbps_whole_node"] = round(nbytes * world * o_steps / el_o / 1e9, 3)
            extra[name + "_ctr_verified"] = v_ok
    if not args.no_aes256:
        v_ok = pdist.allreduce_max(0.0 if verify_once(key256) else 1.0) == 0.0
        k256_steps = max(1, min(args.steps, 5))
        el256, _, _ = timed(k256_steps, key256)
        extra["aes256_ctr_gbps_whole_node"] = round(nbytes * world * k256_steps / el256 / 1e9, 3)
        extra["aes256_ctr_verified"] = v_ok
        extra["aes256_vs_cpu_aesni_ctr256"] = round(extra["aes256_ctr_gbps_whole_node"] / BASELINE_GBPS, 1)
    if not args.no_aes256 and not cpu:
        # AES-256 ECB encryption, in place on the same shard: the reference's
        # own GPU workload (aes-gpu/Source/main_ecb_e.cu) at this scale --
        # "auto" runs the co-resident T-table + bitsliced split here
        def ecb_step(k, impl):
            ops.ecb_encrypt(buf, k, out=buf, impl=impl)

        head, tail = buf[:S].cpu().numpy().tobytes(), buf[nbytes - S:].cpu().numpy().tobytes()
        ecb_step(key256, args.impl)
        sync()
        e_ok = (buf[:S].cpu().numpy().tobytes() == cpu_ref.ecb(key256, head)
                and buf[nbytes - S:].cpu().numpy().tobytes() == cpu_ref.ecb(key256, tail))
        e_ok = pdist.allreduce_max(0.0 if e_ok else 1.0) == 0.0
        e_steps = max(1, min(args.steps, 5))
        el_e, _, _ = timed(e_steps, key256, fn=ecb_step)
        extra["aes256_ecb_gbps_whole_node"] = round(nbytes * world * e_steps / el_e / 1e9, 3)
        extra["aes256_ecb_verified"] = e_ok
        extra["aes256_ecb_impl"] = ops.pick_impl(args.impl, 256, "ecb", nbytes)

    bad = [k for k in ("ttable_ctr_verified", "bitsliced_ctr_verified", "aes256_ctr_verified", "aes256_ecb_verified")
           if extra.get(k) is False]
    if bad:
        if rank == 0:
            emit({"error": "extra verification failed", "failed": bad, **extra})
        sys.exit(1)

    # The extras run after the headline is measured.  An exception in one of
    # them (a transport error at N > 1, say) is recorded in the line instead
    # of losing the headline; a verification FAILURE still ends the run.
    extras_errors = {}
    # the HIP runtime / RCCL this process runs on: in a torch process the
    # library binds torch's bundled copies (HIP 7.0), in otbench /opt/rocm's
    rt_info = None
    if not cpu:
        from our_tree_amd import _native

        rt_info = _native.runtime_info()

    def final_line() -> dict:
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
                "device": args.device,
            },
            "cycles_per_byte_per_cu": round(cpb, 4),
            "cycles_per_byte_per_cu_at_held_clock": round(cpb_eff, 4) if cpb_eff else None,
            "cycles_per_byte_per_cu_at_mean_gfxclk": round(cpb_mean, 4) if cpb_mean else None,
            "held_clock_ghz": round(clk_ghz, 3) if clk_ghz else None,
            "per_gpu_gbps": round(value / world, 3),
            "per_rank_gbps_min": round(min(d["gbps"] for d in table), 3),
            **energy,
            "per_rank": table,
            "preflight": {"ok": pre["ok"], "seconds": pre["seconds"], "bytes": pre["bytes"],
                          "backend": pre["backend"]},
            "baseline": {"value_gbps": BASELINE_GBPS, "what": "AES-NI CTR-256 1000MiB 8thr (BASELINE.md)",
                         "gpu_headline_gbps": BASELINE_GPU_GBPS},
            "verified_sample": all(d["verified"] for d in table),
            "runtime": rt_info,
            **extra,
        }
        if extras_errors:
            line["extras_errors"] = extras_errors
        return line

    def guarded(name, fn):
        """Run one extra stage.  At N = 1 an exception is recorded in the line
        and the run goes on.  At N > 1 the other ranks may be waiting inside
        this stage's collectives, and a rank that skipped ahead would pair its
        next collective with theirs: so the failing rank ends the run (rank 0
        first emits the line with what was measured and the error; the
        launcher stops the other ranks when one exits non-zero)."""
        try:
            return fn()
        except Exception as e:  # noqa: BLE001 -- reported in the JSON line
            extras_errors[name] = f"{type(e).__name__}: {e}"[:500]
            if world > 1:
                print(json.dumps({"rank": rank, "stage_failed": name, "error": extras_errors[name]}),
                      file=sys.stderr, flush=True)
                if rank == 0:
                    emit({**final_line(), "error": f"extra stage '{name}' failed at N > 1"})
                os._exit(1)
            return None

    if not args.no_stream:
        sp = guarded("stream", lambda: stream_pass(args, key, counter, rank, world, local, my_block0))
        extra.update(sp or {"stream_ctr_verified": None})
        if extra["stream_ctr_verified"] is False:
            if rank == 0:
                emit({"error": "host-streamed CTR verification failed", **extra})
            sys.exit(1)

    sc = None
    if not args.no_scatter:
        from our_tree_amd.parallel import jobs

        # The shard stays allocated: the scatter pass needs only 4 x world x
        # chunk more on the root (16 GiB at N = 8).  (An earlier session saw
        # the pinned row's D2H slow down after a 64 GiB free; the probe
        # tools/free_wipe_probe.py did not reproduce it -- 57 GB/s both ways
        # from 38 ms after the free, profiles/r6/validate_d1/free_wipe.jsonl.
        # The row's loss was the engine's streams on pooled hardware queues:
        # profiles/r6/pipeline/census.jsonl, docs/PERF.md round 6.)
        chunk = (args.scatter_mib << 20) if not cpu else 4096 * 8
        sc = guarded("rccl_scatter", lambda: jobs.cbc_scatter_job(args.scatter_rounds, chunk, key256,
                                                                  bytes(range(0xA0, 0xB0)), sector=4096, device=dev))
    if not args.no_scatter and sc is not None:
        extra["rccl_cbc256_scatter_gbps"] = round(sc["gbps"], 3)
        extra["rccl_ranks"] = sc["ranks"]
        extra["rccl_ranks_verified"] = sc["ranks_verified"]
        extra["rccl_backend"] = sc["backend"]
        extra["rccl_duplex"] = sc["overlap"]  # scatter / gather on two communicators (OTC_DUPLEX=0: one)
        extra["rccl_transport"] = sc["transport"]  # "xgmi" over RCCL at N > 1, "local" at N = 1, gloo: "host"
        extra["rccl_xgmi_bytes_verified"] = sc["xgmi_bytes_verified"]
        extra["rccl_xgmi_bytes_timed"] = sc["xgmi_bytes_timed"]
        extra["rccl_host_bytes_verified"] = sc["host_bytes_verified"]
        extra["rccl_scatter_bytes"] = sc["total_bytes"]
        extra["rccl_scatter_verified"] = sc["verified"]
        if not sc["verified"]:
            if rank == 0:
                emit({"error": "RCCL scatter/gather verification failed", "per_rank_ok": sc["per_rank_ok"], **extra})
            sys.exit(1)

    if not args.no_refmethod:
        from our_tree_amd.utils import refmethod

        if rank == 0:
            extra.update(guarded("refmethod", lambda: refmethod.ecb256_three_ways(device=local))
                         or {"refmethod_verified": None})
        if torch.distributed.is_initialized():
            torch.distributed.barrier()
        if rank == 0 and extra["refmethod_verified"] is False:
            emit({"error": "reference-methodology ECB verification failed", **extra})
            sys.exit(1)

    if rank == 0:
        emit(final_line())
    if meter is not None:
        meter.close()
    if torch.distributed.is_initialized():
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
