#!/bin/bash
# Segment-encryption split: T-table claim kernel with 8-block bursts
# double-buffered (tg8, 92-97 VGPRs) or single-buffered (tg8sb, 60-65: room
# for a bigger bs8 wave), and bs8 with 2-block plaintext bursts (tg8sb_b2);
# base = 4-block double-buffered bursts.  AES-256, 4 GiB, verified, power.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
B="--bits 256 --bytes 4G --inplace --iters 40 --verify"
C="--mode cbc-enc-seg --seg 4096 --impl split $B;--mode cbc-enc-seg --seg 512 --impl split $B;--mode cfb-enc-seg --seg 4096 --impl split $B;--mode cbc-enc-seg --seg 4096 --impl ttable $B"
bash scripts/ab_power.sh ${1:-r5_tt_sb_ab} ${2:-1} "$C" base tg8 tg8sb tg8sb_b2
