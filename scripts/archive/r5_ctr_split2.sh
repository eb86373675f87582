#!/bin/bash
# CTR split with the bitsliced tables built before the fork: does it co-run
# at 64 GiB now, and does it beat the bitsliced kernel alone at AES-256?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=${1:-r5_ctr_split2}
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "ctr_split or routing" > gpurun_out/$O.pytest.log 2>&1 || { tail -30 gpurun_out/$O.pytest.log; exit 1; }
tail -1 gpurun_out/$O.pytest.log
C=""
for cfg in "--bits 256 --bytes 64G --inplace --iters 10" "--bits 256 --bytes 4G --iters 20" "--bits 128 --bytes 64G --inplace --iters 10"; do
    for i in bitslice split; do C="$C;--mode ctr $cfg --impl $i --split-stats"; done
done
bash scripts/ab_power.sh $O 2 "${C#;}" base
