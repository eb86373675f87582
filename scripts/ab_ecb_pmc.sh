#!/bin/bash
# Round-3 session-3 measurement batch (run on the box):
# ECB T-table vs bitsliced crossover at 1/4/64 GiB (AES-128 and AES-256),
# then PMC of the bitsliced CTR bulk kernel (AES-128, AES-256) and ECB.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash scripts/xover.sh "256 128" "1G 4G 64G" ecb xover_ecb.jsonl > /dev/null &&
bash scripts/pmc_bulk.sh pmc_ctr128 "--mode ctr --bits 128" &&
bash scripts/pmc_bulk.sh pmc_ctr256 "--mode ctr --bits 256" &&
bash scripts/pmc_bulk.sh pmc_ecb256 "--mode ecb --bits 256" &&
python3 - <<'PY'
import json
for l in open("gpurun_out/xover_ecb.jsonl"):
    d = json.loads(l)
    print(d["mode"], d["bits"], d["bytes"] >> 30, "GiB", d["impl"], d["gbps"], d.get("held_clock_ghz"))
PY
