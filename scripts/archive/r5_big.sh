#!/bin/bash
# Large calls: co-resident split (base) vs the T-table claim kernel alone
# (nobs: a variant built from a patched copy, bs_wgs_for -> 0), with power.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
C="--mode ecb --bits 256 --bytes 64G --inplace --iters 5 --split-stats --impl split"
C="$C;--mode ecb --bits 256 --bytes 16G --iters 10 --split-stats --impl split"
C="$C;--mode cbc-dec --bits 256 --bytes 16G --iters 10 --split-stats --impl split"
C="$C;--mode cfb-dec --bits 256 --bytes 16G --iters 10 --split-stats --impl split"
C="$C;--mode ecb --bits 128 --bytes 64G --inplace --iters 5 --split-stats --impl split"
bash scripts/ab_power.sh ${1:-r5_big} 2 "$C" base nobs
