#!/bin/bash
# A/B: the default memory pool keeping freed memory (base) vs returning it
# at every sync (nokeep, OTC_POOL_KEEP=0): per-call bitsliced tables and the
# split's counter.  Verified, with power, 2 reps interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
C="--mode ctr --bits 128 --bytes 64G --inplace --impl bitslice --iters 60 --warmup 2"
C="$C;--mode ctr --bits 128 --bytes 4G --inplace --impl bitslice --iters 500 --warmup 20"
C="$C;--mode ecb --bits 256 --bytes 1G --inplace --impl split --iters 1500 --warmup 20"
C="$C;--mode ecb --bits 256 --bytes 4G --inplace --impl split --iters 500 --warmup 20"
bash scripts/ab_power.sh ${1:-r4_poolkeep} 2 "$C" base nokeep
