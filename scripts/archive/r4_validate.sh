#!/bin/bash
# Validation of the current build on one MI355X: the whole GPU test suite,
# the bench line (energy, per-rank table, reference-methodology row, verified
# extras), then the J/GB power probe for the bench's own energy keys to be
# compared with.   gpurun --timeout 1200 -- bash scripts/r4_validate.sh NAME
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r4_validate}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 ||
    { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
keys = ["value", "ms_per_step", "held_clock_ghz", "joules_per_gb", "avg_socket_w_per_gpu", "ppt_residency_max",
        "ttable_ctr_gbps_whole_node", "ttable_ctr_verified", "aes256_ctr_gbps_whole_node", "aes256_ctr_verified",
        "refmethod_ecb256_1000mib_gbps", "pinned_e2e_ecb256_1000mib_gbps", "kernel_only_ecb256_1000mib_gbps",
        "refmethod_verified", "stream_ctr_gbps_whole_node", "rccl_cbc256_scatter_gbps"]
for k in keys:
    print(k, d.get(k))
print("per_rank", d["per_rank"])
PY
bash scripts/power_probe.sh bitslice > $O/power.txt 2>&1 || { tail -5 $O/power.txt; exit 1; }
cp -r gpurun_out/power $O/ 2>/dev/null
tail -2 $O/power.txt
