#!/bin/bash
# Does a co-resident T-table share lower CTR's energy per byte under the power
# cap (as it does for ECB)?  ctr-split = T-table CTR on the head + bitsliced CTR
# on the rest (--share = the bitsliced fraction), verified, with power.
#   gpurun --timeout 900 -- bash scripts/r4_ctr_split.sh NAME
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
B="--bytes 64G --inplace --iters 80 --warmup 2"
C="--mode ctr --bits 128 $B --impl bitslice;--mode ctr --bits 128 $B --impl ttable"
for s in 0.95 0.9 0.85 0.8 0.7; do C="$C;--mode ctr-split --bits 128 $B --share $s"; done
C="$C;--mode ctr --bits 256 $B --impl bitslice"
for s in 0.9 0.8; do C="$C;--mode ctr-split --bits 256 $B --share $s"; done
bash scripts/ab_power.sh ${1:-r4_ctr_split} ${2:-1} "$C" base
