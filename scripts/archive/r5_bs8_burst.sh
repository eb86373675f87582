#!/bin/bash
# (evidence script: the knob it varied was removed from the source after the A/B; see docs/PERF.md round 5)
# bs8 plaintext load bursts (OTC_BS8_BURST 1 / 2 / 4: variants base, b8b2,
# b8b4), bs8 alone and in the split, CBC-enc-seg AES-256, 4 KiB and 512 B
# segments, 4 GiB, verified, with power -> gpurun_out/r5_bs8_burst/ab.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
B="--bits 256 --bytes 4G --inplace --iters 40 --verify"
C="--mode cbc-enc-seg --seg 4096 --impl bitslice $B;--mode cbc-enc-seg --seg 4096 --impl split $B;--mode cbc-enc-seg --seg 512 --impl bitslice $B;--mode cbc-enc-seg --seg 512 --impl split $B;--mode cfb-enc-seg --seg 4096 --impl split $B"
bash scripts/ab_power.sh ${1:-r5_bs8_burst} 1 "$C" base b8b2 b8b4
