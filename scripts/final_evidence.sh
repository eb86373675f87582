#!/bin/bash
# PMC of the bitsliced bulk kernels of the current build (AES-128/256 CTR)
# and a sustained 1000-step bench (held clock + GB/s over ~45 s), on the box:
#   gpurun --timeout 900 -- bash scripts/final_evidence.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash scripts/pmc_bulk.sh pmc_final_ctr128 "--mode ctr --bits 128" &&
bash scripts/pmc_bulk.sh pmc_final_ctr256 "--mode ctr --bits 256" &&
timeout -k 10 300 python bench.py --steps 1000 --warmup 3 --no-aes256 --no-scatter --no-stream --no-other-impl \
    > gpurun_out/sustained_1000.json 2> gpurun_out/sustained_1000.err && cat gpurun_out/sustained_1000.json
