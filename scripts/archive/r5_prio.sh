#!/bin/bash
# (evidence script: the knob it varied was removed from the source after the A/B; see docs/PERF.md round 5)
# Co-resident split (base) vs the T-table claim kernel alone (nobs) vs the
# split with the T-table waves at issue priority 3 (prio3): AES-256 4 GiB.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
B="--bits ${BITS:-256} --bytes 4G --iters ${ITERS:-30} --split-stats --impl split"
C="--mode ecb $B;--mode cbc-dec $B;--mode cfb-dec $B;--mode cbc-enc-seg --seg 4096 $B;--mode cbc-enc-seg --seg 512 $B"
bash scripts/ab_power.sh ${1:-r5_prio} 1 "$C" ${VARIANTS:-base nobs prio3}
