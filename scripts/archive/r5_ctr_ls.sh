#!/bin/bash
# (evidence script: the CTR split it measures was not adopted; its source is profiles/r5/ctr_split/ctr_split.patch)
# CTR split: LDS staging slots of the bitsliced CTR claim kernel (4 = base, 6)
# -- does it co-reside beside the 128 KiB T-table? (split_units: both > 0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
C="--mode ctr --bits 128 --bytes 64G --inplace --iters 10 --impl split --split-stats;--mode ctr --bits 128 --bytes 4G --iters 20 --impl split --split-stats;--mode ctr --bits 128 --bytes 64G --inplace --iters 10 --impl bitslice"
bash scripts/ab_power.sh ${1:-r5_ctr_ls} 2 "$C" base ls6
