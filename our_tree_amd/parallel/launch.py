"""Self-launch of one process per GPU without torchrun.

``python bench.py --gpus 8`` must measure 8 GPUs whether or not a launcher set
RANK/WORLD_SIZE.  The decision is made BEFORE anything touches the GPU (no HIP
call, no ``torch.cuda.is_available()``, no native library load): counting
devices with ``torch.cuda.device_count()`` does not initialise HIP on this
image, everything else does, and a process that has initialised the GPU must
not fork children that use it.

Plan (``plan_launch``):

* a launcher already set ``WORLD_SIZE``: it must equal ``--gpus`` (a mismatch
  is an error -- never silently measure a different number of GPUs);
* ``--gpus 1`` and no launcher: run in this process;
* ``--gpus N > 1`` and no launcher: spawn N fresh interpreters (RANK /
  LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / a free MASTER_PORT), relay
  their output, exit with the first failing child's code.  Fewer than N
  visible GPUs is an error unless ``OTC_SHARE_GPUS=1`` (rehearsal: several
  ranks share one device, gloo backend).

The reference's scaling sweep ran {1,2,4,8} pthreads inside one process
(/root/reference/test.c:135-153, aes-modes/test.c:422-440); here the workers
are processes, one per GPU, talking RCCL over xGMI.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import threading
import time
from dataclasses import dataclass

LAUNCH_VARS = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


@dataclass(frozen=True)
class LaunchPlan:
    action: str          # "run" | "spawn" | "error"
    nprocs: int = 1
    message: str = ""


def visible_gpus() -> int:
    """Device count without initialising HIP (torch.cuda.device_count reads
    the driver's device list only); 0 when torch has no ROCm build."""
    try:
        import torch

        return int(torch.cuda.device_count())
    except Exception:  # pragma: no cover - torch always importable here
        return 0


def plan_launch(gpus: int, env: dict | None = None, ndev: int | None = None) -> LaunchPlan:
    env = os.environ if env is None else env
    if gpus < 1:
        return LaunchPlan("error", message=f"--gpus must be >= 1 (got {gpus})")
    share = env.get("OTC_SHARE_GPUS") == "1"
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            return LaunchPlan("error", message=f"--gpus {gpus} but the launcher set WORLD_SIZE={world}; "
                                                "refusing to measure a different number of GPUs")
        return LaunchPlan("run", world)
    if gpus == 1:
        return LaunchPlan("run", 1)
    n = visible_gpus() if ndev is None else ndev
    if n < gpus and not share:
        return LaunchPlan("error", message=f"--gpus {gpus} requested but only {n} GPU(s) are visible "
                                            "(OTC_SHARE_GPUS=1 rehearses several ranks on one device)")
    return LaunchPlan("spawn", gpus)


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def child_env(rank: int, world: int, port: int, base: dict | None = None) -> dict:
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
    return env


def _child_setup(parent_pid: int):
    """Runs in the forked child before it execs the worker (nothing has touched
    the GPU in this launcher, so the exec is safe): ask the kernel to SIGTERM
    the child when the launcher dies, however it dies -- a SIGKILL of the
    launcher leaves no orphaned rank holding a GPU.  If the launcher is
    already gone (the race before prctl), exit at once."""
    try:
        import ctypes

        libc = ctypes.CDLL("libc.so.6", use_errno=True)
        libc.prctl(1, int(signal.SIGTERM), 0, 0, 0)  # PR_SET_PDEATHSIG
    except Exception:  # pragma: no cover - non-Linux
        pass
    if os.getppid() != parent_pid:
        os._exit(1)


def spawn(nprocs: int, argv: list[str], timeout_s: float | None = None, grace_s: float = 10.0) -> int:
    """Start ``nprocs`` copies of ``argv`` (one per rank) and wait.  Children
    share this process's stdout/stderr.  When one fails, the others are
    terminated (by PID -- they are our own children) and its exit code is
    returned.

    Kill safety: every child gets a parent-death signal (``_child_setup``);
    SIGTERM / SIGINT / SIGHUP sent to the launcher are forwarded to the
    children, which get ``grace_s`` seconds to exit before SIGKILL; after
    ``timeout_s`` the children are terminated the same way (exit code 124)."""
    port = free_port()
    me = os.getpid()
    procs: list = []
    got = []

    def _fg_group() -> bool:
        """the launcher's process group owns the terminal: a terminal ^C
        already reached every child (they share the group)"""
        try:
            return os.tcgetpgrp(sys.stdin.fileno()) == os.getpgrp()
        except (OSError, ValueError, AttributeError):
            return False

    def on_signal(signum, frame):
        got.append(signum)
        if signum == signal.SIGINT and _fg_group():
            return  # a second SIGINT would cut the ranks' own cleanup short
        for p in procs:
            if p.poll() is None:
                p.send_signal(signum)

    handled = (signal.SIGTERM, signal.SIGINT, signal.SIGHUP)
    old = {}
    t0 = time.monotonic()
    rc = 0
    stop_at = None  # monotonic deadline for SIGKILL after a terminate
    try:
        # handlers first (inside the try: whatever fails, the finally below
        # stops every child that was started); signal.signal works on the
        # main thread only -- elsewhere the children rely on the finally and
        # their parent-death signal
        if threading.current_thread() is threading.main_thread():
            old = {s_: signal.signal(s_, on_signal) for s_ in handled}
        for r in range(nprocs):
            procs.append(subprocess.Popen(argv, env=child_env(r, nprocs, port),
                                          preexec_fn=lambda: _child_setup(me)))
        live = set(range(nprocs))
        while live:
            for r in sorted(live):
                c = procs[r].poll()
                if c is None:
                    continue
                live.discard(r)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    if not got:
                        print(f"launch: rank {r} exited with {c}; stopping the other ranks", file=sys.stderr)
                    for q in live:
                        procs[q].send_signal(signal.SIGTERM)
                    stop_at = stop_at or time.monotonic() + grace_s
            if got and stop_at is None:
                stop_at = time.monotonic() + grace_s
            if timeout_s is not None and time.monotonic() - t0 > timeout_s and live and stop_at is None:
                print(f"launch: timeout after {timeout_s:.0f} s; stopping the ranks", file=sys.stderr)
                for q in live:
                    procs[q].send_signal(signal.SIGTERM)
                rc = rc or 124
                stop_at = time.monotonic() + grace_s
            if stop_at is not None and time.monotonic() > stop_at:
                for q in live:
                    procs[q].kill()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        for s_, h in old.items():
            signal.signal(s_, h)
    if got and rc == 0:
        rc = 128 + int(got[0])
    return rc


def dispatch(gpus: int, script: str, argv: list[str], timeout_s: float | None = None) -> bool:
    """Apply the plan for a script run as ``python script argv``.  Returns True
    when the caller should run its main body in this process; otherwise exits
    (spawned run finished, or refused).  ``timeout_s`` bounds a spawned run."""
    p = plan_launch(gpus)
    if p.action == "run":
        return True
    if p.action == "error":
        print(f"error: {p.message}", file=sys.stderr)
        sys.exit(2)
    sys.exit(spawn(p.nprocs, [sys.executable, script] + list(argv), timeout_s=timeout_s))
