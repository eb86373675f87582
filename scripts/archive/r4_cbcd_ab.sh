#!/bin/bash
# A/B: CBC-decrypt bitsliced output-phase lookahead 4 (base) vs 2 (cbcd2),
# through the split, the segment split and the bitsliced kernel alone.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
B="--bits 256 --iters 100 --warmup 3"
C="--mode cbc-dec $B --bytes 32G --impl split;--mode cbc-dec-seg $B --bytes 16G --seg 4096 --impl split"
C="$C;--mode cbc-dec $B --bytes 16G --impl bitslice"
bash scripts/ab_power.sh ${1:-r4_cbcd_ab} 2 "$C" base cbcd2
