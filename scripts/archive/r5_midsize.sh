#!/bin/bash
# [896 MiB, 2 GiB): persistent T-table claim kernel alone (base) vs the grid
# T-table kernel (variant grid), impl auto, 2 reps, with power; + GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py > gpurun_out/r5_midsize.pytest.log 2>&1 || { tail -30 gpurun_out/r5_midsize.pytest.log; exit 1; }
tail -1 gpurun_out/r5_midsize.pytest.log
C=""
for cfg in "ecb --bits 256 --bytes 1000M" "ecb-dec --bits 256 --bytes 1000M" "cbc-dec --bits 256 --bytes 1000M" "cfb-dec --bits 256 --bytes 1000M" \
           "ecb --bits 128 --bytes 1000M" "ecb --bits 256 --bytes 1536M" "cbc-dec --bits 256 --bytes 1536M" "cbc-dec --bits 128 --bytes 1G"; do
    C="$C;--mode $cfg --iters 30 --split-stats"
done
bash scripts/ab_power.sh ${1:-r5_midsize} 2 "${C#;}" base grid
