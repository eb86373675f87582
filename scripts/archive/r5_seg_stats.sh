#!/bin/bash
# Segment-encryption split with the units each side took (--split-stats),
# one or two bs8 workgroups per CU (base, w2), AES-256 / AES-128, 4 KiB and
# 512 B segments, 4 and 32 GiB; verified, with power.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
B="--inplace --iters ${ITERS:-40} --verify --split-stats"
C="--mode cbc-enc-seg --bits 256 --bytes 4G --seg 4096 --impl split $B;--mode cbc-enc-seg --bits 256 --bytes 4G --seg 512 --impl split $B;--mode cfb-enc-seg --bits 256 --bytes 4G --seg 4096 --impl split $B;--mode cbc-enc-seg --bits 128 --bytes 4G --seg 4096 --impl split $B"
bash scripts/ab_power.sh ${1:-r5_seg_stats} 1 "$C" ${VARIANTS:-base w2}
