#!/bin/bash
# The split modes after moving both halves to CU-masked streams (otbench,
# null stream): do the round-5 numbers hold?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
C="--mode ecb --bits 256 --bytes 64G --inplace --iters 10 --split-stats;--mode cbc-dec --bits 256 --bytes 16G --iters 10 --split-stats;--mode cfb-dec --bits 256 --bytes 16G --iters 10 --split-stats;--mode ecb --bits 128 --bytes 4G --iters 20 --split-stats;--mode cbc-enc-seg --bits 256 --seg 4096 --bytes 32G --inplace --iters 6 --split-stats"
bash scripts/ab_power.sh ${1:-r5_cumask} ${REPS:-1} "$C" ${VARIANTS:-base}
