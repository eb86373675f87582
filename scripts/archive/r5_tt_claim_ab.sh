#!/bin/bash
# (evidence script: the knob it varied was removed from the source after the A/B; see docs/PERF.md round 5)
# T-table half of the segment-encryption split: 4- vs 8-block bursts
# (OTC_SEG_CLAIM_G; base = 4, tg8 = 8) and non-temporal plaintext /
# ciphertext (OTC_SEG_TT_NT; ttnt, tg8nt), CBC-enc-seg AES-256, 4 GiB,
# 4 KiB / 512 B segments, split; verified, with power.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
B="--bits 256 --bytes 4G --inplace --iters 40 --verify"
C="--mode cbc-enc-seg --seg 4096 --impl split $B;--mode cbc-enc-seg --seg 512 --impl split $B;--mode cbc-enc-seg --seg 4096 --impl ttable $B"
bash scripts/ab_power.sh ${1:-r5_tt_claim_ab} 1 "$C" base tg8 ttnt tg8nt
