"""bench.py launch contract (parallel/launch.py), on CPU.

``python bench.py --gpus N`` must run N ranks or fail loudly: never measure a
different number of GPUs than asked.  The plan is made
before any GPU call; spawned ranks get RANK/LOCAL_RANK/WORLD_SIZE and a
127.0.0.1 rendezvous."""
import json
import os
import subprocess
import sys

import pytest

from our_tree_amd.parallel import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("gpus,env,ndev,action", [
    (1, {}, 0, "run"),
    (1, {}, 8, "run"),
    (8, {}, 8, "spawn"),
    (4, {}, 8, "spawn"),
    (2, {}, 1, "error"),
    (8, {}, 0, "error"),
    (2, {"OTC_SHARE_GPUS": "1"}, 1, "spawn"),
    (8, {"WORLD_SIZE": "8"}, 8, "run"),
    (8, {"WORLD_SIZE": "1"}, 8, "error"),
    (1, {"WORLD_SIZE": "2"}, 8, "error"),
    (0, {}, 8, "error"),
])
def test_plan(gpus, env, ndev, action):
    p = launch.plan_launch(gpus, env=env, ndev=ndev)
    assert p.action == action, p
    if action == "spawn":
        assert p.nprocs == gpus
    if action == "error":
        assert p.message


def test_child_env():
    e = launch.child_env(3, 8, 12345, base={"FOO": "1"})
    assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"]) == ("3", "3", "8")
    assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "12345" and e["FOO"] == "1"


def test_spawn_runs_every_rank(tmp_path):
    script = tmp_path / "w.py"
    out = tmp_path / "out"
    out.mkdir()
    script.write_text(
        "import os, sys\n"
        f"open(os.path.join({str(out)!r}, os.environ['RANK']), 'w').write(os.environ['WORLD_SIZE'] + ' ' + "
        "os.environ['MASTER_ADDR'] + ' ' + ' '.join(sys.argv[1:]))\n")
    rc = launch.spawn(4, [sys.executable, str(script), "--x", "1"], timeout_s=60)
    assert rc == 0
    assert sorted(os.listdir(out)) == ["0", "1", "2", "3"]
    for r in range(4):
        assert (out / str(r)).read_text() == "4 127.0.0.1 --x 1"


def test_spawn_propagates_failure(tmp_path):
    script = tmp_path / "w.py"
    script.write_text("import os, sys, time\n"
                      "if os.environ['RANK'] == '1': sys.exit(7)\n"
                      "time.sleep(30)\n")
    rc = launch.spawn(3, [sys.executable, str(script)], timeout_s=60)
    assert rc == 7


def _bench(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in launch.LAUNCH_VARS and k != "OTC_SHARE_GPUS"}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=300, env=env, cwd=ROOT)


def test_bench_refuses_more_gpus_than_visible():
    import torch

    n = torch.cuda.device_count()
    r = _bench(["--gpus", str(max(2, n + 1)), "--steps", "1", "--warmup", "0"])
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "GPU(s) are visible" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_bench_refuses_world_size_mismatch():
    r = _bench(["--gpus", "2", "--steps", "1"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2, r.stderr[-2000:]
    assert "WORLD_SIZE=1" in r.stderr


# ---- kill safety ---------------------------
_LAUNCHER = (
    "import sys; sys.path.insert(0, {root!r})\n"
    "from our_tree_amd.parallel import launch\n"
    "sys.exit(launch.spawn(3, [sys.executable, {child!r}], timeout_s={timeout}, grace_s=2))\n")
_CHILD = ("import os, time\n"
          "open(os.path.join({d!r}, os.environ['RANK']), 'w').write(str(os.getpid()))\n"
          "time.sleep(120)\n")


def _alive(pid):
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split(")")[-1].split()[0] != "Z"
    except FileNotFoundError:
        return False


def _start_launcher(tmp_path, timeout="None"):
    import time

    d = tmp_path / "pids"
    d.mkdir()
    child = tmp_path / "child.py"
    child.write_text(_CHILD.format(d=str(d)))
    p = subprocess.Popen([sys.executable, "-c", _LAUNCHER.format(root=ROOT, child=str(child), timeout=timeout)])
    t0 = time.time()
    while len(os.listdir(d)) < 3 and time.time() - t0 < 60:
        time.sleep(0.1)
    time.sleep(0.3)  # let the pid files be written completely
    pids = [int((d / f).read_text()) for f in sorted(os.listdir(d))]
    assert len(pids) == 3 and all(_alive(q) for q in pids)
    return p, pids


def _wait_gone(pids, limit=15.0):
    import time

    t0 = time.time()
    while any(_alive(q) for q in pids) and time.time() - t0 < limit:
        time.sleep(0.1)
    return [q for q in pids if _alive(q)]


def test_killed_launcher_leaves_no_rank(tmp_path):
    """SIGKILL of the launcher (no handler can run): the parent-death signal
    ends every rank"""
    import signal

    p, pids = _start_launcher(tmp_path)
    p.send_signal(signal.SIGKILL)
    p.wait(timeout=10)
    assert _wait_gone(pids) == []


def test_sigterm_is_forwarded(tmp_path):
    import signal

    p, pids = _start_launcher(tmp_path)
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=20) == 128 + signal.SIGTERM
    assert _wait_gone(pids) == []


def test_spawn_timeout_stops_ranks(tmp_path):
    p, pids = _start_launcher(tmp_path, timeout="8")
    assert p.wait(timeout=30) == 124
    assert _wait_gone(pids) == []


@pytest.mark.parametrize("script", ["benchmarks/cbc_scatter.py", "benchmarks/stream_ctr.py"])
def test_config_benchmarks_refuse_more_gpus_than_visible(script):
    """configs 4 and 5 take --gpus N like bench.py: self-spawned, or refused
    on a box with fewer GPUs (OTC_SHARE_GPUS=1 rehearses)"""
    import torch

    n = torch.cuda.device_count()
    env = {k: v for k, v in os.environ.items() if k not in launch.LAUNCH_VARS and k != "OTC_SHARE_GPUS"}
    r = subprocess.run([sys.executable, os.path.join(ROOT, script), "--gpus", str(max(2, n + 1))],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "GPU(s) are visible" in r.stderr
