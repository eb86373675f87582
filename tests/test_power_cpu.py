"""tools/power_run.py and utils/power.PowerMeter without a GPU: the wrapper
passes the command's JSON through, extended with the power record (here
"unavailable", no amdsmi device in the container) and the marks' wall time,
and never initialises HIP itself (torch_bdf=False)."""
import json
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_power_run_wraps_marks(tmp_path):
    child = tmp_path / "child.py"
    child.write_text(textwrap.dedent("""
        import sys, time, json
        print("OTB_MARK start", file=sys.stderr, flush=True)
        time.sleep(0.3)
        print("OTB_MARK end", file=sys.stderr, flush=True)
        print("some log line", file=sys.stderr)
        print(json.dumps({"mode": "ecb", "bytes": 1 << 20, "iters": 10, "ms": 30.0, "gbps": 1.0}))
    """))
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "power_run.py"), "--label", "x", "--",
                        sys.executable, str(child)], capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert p.returncode == 0, p.stderr
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["label"] == "x" and d["mode"] == "ecb"
    assert 0.25 < d["marks_wall_s"] < 5
    assert "power" in d
    if not d["power"].get("available"):
        assert d["power"]["reason"]
    assert "some log line" in p.stderr


def test_meter_without_torch_does_not_import_torch():
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from our_tree_amd.utils.power import PowerMeter\n"
            "m = PowerMeter(0, torch_bdf=False); m.start(); s = m.stop()\n"
            "assert 'torch' not in sys.modules, 'torch imported'\n"
            "print(s.get('available'))\n") % ROOT
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
