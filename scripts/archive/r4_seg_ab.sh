#!/bin/bash
# A/B of the grouped CBC / CFB segment-encryption kernel: 1 segment per lane
# with 8-block bursts (base) vs 2 segments per lane (more independent chains
# for the LDS latency) with 4- or 8-block bursts.  Verified, with power.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
B="--bytes 4G --inplace --iters 600 --warmup 20"
C="--mode cbc-enc-seg --bits 256 $B;--mode cfb-enc-seg --bits 256 $B;--mode cbc-enc-seg --bits 128 $B"
bash scripts/ab_power.sh ${1:-r4_seg_ab} 2 "$C" base segb2g4 segb2g8
