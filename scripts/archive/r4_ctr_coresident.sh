#!/bin/bash
# Is there a co-residency gain for CTR?  The T-table CTR kernel at B=4 takes
# 111-113 registers (no bitsliced wave fits beside it); variant ctrb2 (B=2)
# leaves room for one.  Static ctr-split (joined per call) at high bitsliced
# shares, both variants, verified, with power.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
B="--bytes 64G --inplace --iters 80 --warmup 2"
C="--mode ctr --bits 128 $B --impl bitslice;--mode ctr --bits 128 $B --impl ttable"
for s in 0.95 0.9 0.85 0.8; do C="$C;--mode ctr-split --bits 128 $B --share $s"; done
bash scripts/ab_power.sh ${1:-r4_ctr_cores} 1 "$C" base ctrb2
