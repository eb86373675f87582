"""bench.py driver contract: one JSON line with the fields the round driver
reads (metric/value/unit/n_gpus/steps/warmup/ms_per_step/...), the metric and
config BASELINE.json names, and value consistent with ms_per_step.

The GPU test runs the real headline step on a small shard (0.25 GiB instead of
64 GiB, so it finishes in seconds); the CPU test only checks the CLI surface."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config")


def test_bench_cli_help():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--help"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    for flag in ("--gpus", "--steps", "--warmup"):
        assert flag in r.stdout


def test_baseline_ratios_are_labelled():
    """vs_baseline divides AES-128-CTR bytes by the AES-256 CPU headline and
    says so; the AES-128-equivalent ratio uses the 14/10 round ratio
    """
    sys.path.insert(0, ROOT)
    import bench

    r = bench.baseline_ratios(1519.0)
    assert bench.BASELINE_GBPS == 0.519
    assert r["vs_baseline"] == pytest.approx(1519.0 / 0.519, rel=1e-3)
    assert "AES-128" in r["vs_baseline_what"] and "CTR-256" in r["vs_baseline_what"]
    assert "results.frankchn.aesni:32" in r["vs_baseline_what"]
    assert r["vs_baseline_aes128_equiv"] == pytest.approx(1519.0 / (0.519 * 1.4), rel=1e-3)


@pytest.mark.gpu
def test_bench_json_line(gpu):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--gib", "0.25", "--no-clock", "--no-aes256", "--no-other-impl",
                        "--scatter-mib", "64", "--scatter-rounds", "2", "--stream-gib", "0.25",
                        "--stream-passes", "2"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    # stdout is the one JSON line and nothing else (RCCL's banner goes to stderr)
    lines = r.stdout.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout
    d = json.loads(lines[0])
    for k in REQUIRED:
        assert k in d, k
    assert d["metric"] == "GB/s AES-128-CTR (whole node)"
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["config"]["model"] == "AES-128-CTR" and d["config"]["parallelism"] == "dp1"
    assert d["verified_sample"] is True
    assert d["config"]["impl_resolved"] == "ttable"  # 0.25 GiB: below the bitsliced threshold
    nbytes = d["config"]["per_gpu_bytes"]
    assert nbytes == int(0.25 * (1 << 30))
    # value (GB/s) and ms_per_step describe the same timed region
    assert d["value"] == pytest.approx(nbytes / (d["ms_per_step"] * 1e-3) / 1e9, rel=0.01)
    assert d["value"] > 100.0  # the HIP kernel ran (an eager fallback would be far slower)
    # the communication pass ran through a (1-rank) RCCL group and verified
    assert d["rccl_ranks"] == 1 and d["rccl_backend"] == "nccl"
    assert d["rccl_scatter_verified"] is True and d["rccl_cbc256_scatter_gbps"] > 0
    assert d["rccl_ranks_verified"] == 1
    assert d["rccl_xgmi_bytes_verified"] == 0 and d["rccl_xgmi_bytes_timed"] == 0  # 1 rank: nothing crosses
    assert "vs_baseline_what" in d and d["vs_baseline_aes128_equiv"] < d["vs_baseline"]
    # host-streamed pass: verified, every rank's NUMA node and PCIe rates
    assert d["stream_ctr_verified"] is True and d["stream_ctr_gbps_whole_node"] > 5
    assert d["stream_ctr_bytes_per_rank"] == 2 * int(0.25 * (1 << 30))
    pr = d["stream_ctr_per_rank"]
    assert len(pr) == 1 and pr[0]["rank"] == 0 and pr[0]["h2d_gbps"] > 0 and pr[0]["d2h_gbps"] > 0
