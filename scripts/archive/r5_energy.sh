#!/bin/bash
# Round-5 per-kernel energy table: every mode at impl auto (what a user
# gets), verified, socket energy over the timed loop (tools/power_run.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
C="--mode ctr --bits 128 --bytes 64G --inplace --iters 10"
C="$C;--mode ctr --bits 256 --bytes 64G --inplace --iters 10"
C="$C;--mode ecb --bits 128 --bytes 64G --inplace --iters 10"
C="$C;--mode ecb --bits 256 --bytes 64G --inplace --iters 10"
C="$C;--mode ecb-dec --bits 256 --bytes 32G --iters 10"
C="$C;--mode cbc-dec --bits 256 --bytes 32G --iters 10"
C="$C;--mode cfb-dec --bits 256 --bytes 32G --iters 10"
C="$C;--mode cbc-enc-seg --bits 256 --seg 4096 --bytes 32G --inplace --iters 6"
C="$C;--mode cfb-enc-seg --bits 256 --seg 4096 --bytes 32G --inplace --iters 6"
C="$C;--mode cbc-enc-seg --bits 256 --seg 512 --bytes 32G --inplace --iters 6"
C="$C;--mode cbc-dec-seg --bits 256 --seg 4096 --bytes 32G --iters 10"
C="$C;--mode cfb-dec-seg --bits 256 --seg 4096 --bytes 32G --iters 10"
C="$C;--mode cbc-enc-seg --bits 128 --seg 4096 --bytes 32G --inplace --iters 6"
C="$C;--mode cbc-dec --bits 128 --bytes 32G --iters 10"
C="$C;--mode rc4 --streams 131072 --len 8K --iters 10"
C="$C;--mode rc4 --streams 1M --len 1K --iters 10"
bash scripts/ab_power.sh ${1:-r5_energy} 1 "$C" base
