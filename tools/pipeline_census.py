#!/usr/bin/env python3
"""Where the pinned end-to-end pipeline loses its overlap.

One process walks through the states bench.py's process passes through and,
after each, times the pinned 3-stream pipeline (AES-256 ECB, 1000 MiB, 64 MiB
chunks, key setup inside the timer -- utils/refmethod.py's "pinned" row) with
the engine's streams on HIP's pooled hardware queues and on queues of their
own (otc_engine_create_ex).  Each record carries the per-phase event sums
(H2D / kernel / D2H ms), the overlap ratio wall / (h2d + kernel + d2h), the
process's KFD queue census (/sys/class/kfd/kfd/proc/<pid>/queues, when
readable) and the runtime the library is bound to.

States:  torch   torch.cuda initialised, nothing else
         nccl    + a 1-rank RCCL process group (one all_reduce)
         split   + an AES-256 ECB split call (two CU-masked auxiliary streams)
         scatter + jobs.cbc_scatter_job (bench.py's RCCL pass: two more communicators)
         busy    + 12 torch streams with kernels queued on them while timing

Usage: python tools/pipeline_census.py [--iters 10] [--out FILE]
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


def kfd_queues() -> dict:
    """Count this process's user-mode queues by type (KFD sysfs)."""
    base = f"/sys/class/kfd/kfd/proc/{os.getpid()}/queues"
    out: dict = {}
    try:
        for q in os.listdir(base):
            try:
                with open(os.path.join(base, q, "type")) as f:
                    t = f.read().strip()
            except OSError:
                t = "?"
            out[t] = out.get(t, 0) + 1
    except OSError as e:
        return {"unreadable": str(e)[:80]}
    return out


_SPIN = {}


def spin_cycles(seconds: float) -> int:
    """torch.cuda._sleep argument that spins ~``seconds`` (calibrated once)."""
    if "per_s" not in _SPIN:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda._sleep(10_000_000)
        torch.cuda.synchronize()
        _SPIN["per_s"] = 10_000_000 / max(time.perf_counter() - t0, 1e-6)
    return int(_SPIN["per_s"] * seconds)


def pinned_pass(pin_in, pin_out, key, iters, pooled, device=0, before_iter=None) -> dict:
    from our_tree_amd.parallel import stream as pstream

    with pstream.StreamEngine(device, chunk_bytes=64 << 20, depth=3, pooled_queues=pooled) as eng:
        eng.run("ecb", pin_in, pin_out, key)
        walls, h2d, k, d2h = [], 0.0, 0.0, 0.0
        for _ in range(iters):
            if before_iter:
                before_iter()
            t0 = time.perf_counter()
            st = eng.run("ecb", pin_in, pin_out, key)
            walls.append(time.perf_counter() - t0)
            h2d += st["h2d_ms"] / iters
            k += st["kernel_ms"] / iters
            d2h += st["d2h_ms"] / iters
        census = kfd_queues()
    n = pin_in.size
    wall = sum(walls) / len(walls)
    return {"gbps": round(n / wall / 1e9, 2), "gbps_best": round(n / min(walls) / 1e9, 2),
            "wall_ms": round(wall * 1e3, 2), "h2d_ms": round(h2d, 2), "kernel_ms": round(k, 2),
            "d2h_ms": round(d2h, 2), "overlap_ratio": round(wall * 1e3 / (h2d + k + d2h), 3),
            "kfd_queues_during": census}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--mib", type=int, default=1000)
    ap.add_argument("--out", default=None)
    ap.add_argument("--states", default="torch,nccl,split,scatter,busy")
    ap.add_argument("--realloc", action="store_true",
                    help="allocate the pinned buffers afresh after every state (as refmethod does)")
    args = ap.parse_args()

    from our_tree_amd import _native, ops
    from our_tree_amd.models import cpu_ref
    from our_tree_amd.parallel import stream as pstream

    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda").sum().item()
    lib = _native.require_gpu_lib()
    rt = _native.runtime_info()
    nbytes = args.mib << 20
    rng = np.random.default_rng(1)
    key = bytes(rng.integers(0, 256, 32, dtype=np.uint8).tolist())
    pin_in, pin_out = pstream.pinned_empty(nbytes), pstream.pinned_empty(nbytes)
    pin_in[:] = rng.integers(0, 256, nbytes, dtype=np.uint8)
    outf = open(args.out, "a") if args.out else None

    def emit(rec):
        line = json.dumps(rec)
        print(line, flush=True)
        if outf:
            outf.write(line + "\n")
            outf.flush()

    emit({"runtime": rt, "kfd_queues_start": kfd_queues()})
    busy_streams = []
    for state in args.states.split(","):
        if state == "nccl":
            from our_tree_amd.parallel import dist as pdist

            pdist.init_from_env(force=True)
            t = torch.ones(1, device="cuda")
            torch.distributed.all_reduce(t)
            torch.cuda.synchronize()
        elif state == "split":
            x = torch.empty(4 << 30, dtype=torch.uint8, device="cuda")
            ops.fill_random_(x, seed=3)
            ops.ecb_encrypt(x, key, out=x)
            torch.cuda.synchronize()
            emit({"state": state, "split_impl": ops.last_impl()})
            del x
            torch.cuda.empty_cache()
        elif state == "scatter":
            from our_tree_amd.parallel import jobs

            sc = jobs.cbc_scatter_job(4, 512 << 20, key, bytes(range(0xA0, 0xB0)), sector=4096,
                                      device=torch.device("cuda", 0))
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            emit({"state": state, "scatter_gbps": round(sc["gbps"], 2), "verified": sc["verified"]})
        elif state == "busy" and not busy_streams:
            busy_streams = [torch.cuda.Stream() for _ in range(12)]
        if args.realloc:
            del pin_in, pin_out
            pin_in, pin_out = pstream.pinned_empty(nbytes), pstream.pinned_empty(nbytes)
            pin_in[:] = rng.integers(0, 256, nbytes, dtype=np.uint8)
        emit({"state": state, "pinned_numa_nodes": [lib.otc_numa_node_of_addr(a.ctypes.data) for a in (pin_in, pin_out)],
              "affinity_cpus": len(os.sched_getaffinity(0)),
              "affinity_first": sorted(os.sched_getaffinity(0))[:4], "threads": len(os.listdir("/proc/self/task")),
              "gpu_numa_node": lib.otc_device_numa_node(0)})
        for pooled in (True, False):
            busy = None
            if state == "busy":
                # before every timed iteration each busy stream gets one
                # one-wave spin kernel as long as a pipeline pass (~25 ms): a
                # pooled queue shared with one of them holds the pipeline's
                # work behind it; a queue of its own does not
                cyc = spin_cycles(0.025)

                def busy():
                    for s in busy_streams:
                        with torch.cuda.stream(s):
                            torch.cuda._sleep(cyc)
            r = pinned_pass(pin_in, pin_out, key, args.iters, pooled, before_iter=busy)
            ok = (pin_out[:65536].tobytes() == cpu_ref.ecb(key, pin_in[:65536].tobytes())
                  and pin_out[-65536:].tobytes() == cpu_ref.ecb(key, pin_in[-65536:].tobytes()))
            emit({"state": state, "queues": "pooled" if pooled else "dedicated", "verified": ok, **r,
                  "kfd_queues_after": kfd_queues()})
            if state == "busy":
                torch.cuda.synchronize()
    lib.otc_release_resources()
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
