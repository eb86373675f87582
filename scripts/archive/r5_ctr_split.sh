#!/bin/bash
# (evidence script: the CTR split it measures was not adopted; its source is profiles/r5/ctr_split/ctr_split.patch)
# CTR as a co-resident split (bitsliced CTR claim + T-table CTR claim) vs the
# bitsliced kernel alone (the headline path) vs the T-table: AES-128 / 256,
# 64 GiB in place (the headline shape) and 4 GiB, with power.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=${1:-r5_ctr_split}
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "ctr_split or routing" > gpurun_out/$O.pytest.log 2>&1 || { tail -30 gpurun_out/$O.pytest.log; exit 1; }
tail -2 gpurun_out/$O.pytest.log
C=""
for cfg in "--bits 128 --bytes 64G --inplace --iters 10" "--bits 256 --bytes 64G --inplace --iters 10" "--bits 128 --bytes 4G --iters 20"; do
    for i in bitslice split ttable; do C="$C;--mode ctr $cfg --impl $i --split-stats"; done
done
bash scripts/ab_power.sh $O ${REPS:-2} "${C#;}" base
