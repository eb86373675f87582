#!/bin/bash
# A/B: the claimed split with 4 T-table waves x 4 (or 2) blocks + 1 bitsliced
# wave per SIMD (base) vs 4 T-table waves x 1 block + 2 bitsliced waves per
# SIMD (claimb1: T-table claim kernels at 40-ish registers, 2 bitsliced
# claim workgroups per CU).  Verified, with power.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
C="--mode ecb --bits 256 --bytes 64G --inplace --impl split --iters 60 --warmup 2"
C="$C;--mode ecb --bits 256 --bytes 4G --inplace --impl split --iters 600 --warmup 20"
C="$C;--mode ecb-dec --bits 256 --bytes 64G --inplace --impl split --iters 60 --warmup 2"
C="$C;--mode cbc-dec --bits 256 --bytes 32G --impl split --iters 100 --warmup 2"
C="$C;--mode ecb --bits 128 --bytes 64G --inplace --impl split --iters 60 --warmup 2"
bash scripts/ab_power.sh ${1:-r4_claimb1_ab} 2 "$C" base claimb1
