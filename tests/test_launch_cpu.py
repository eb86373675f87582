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
