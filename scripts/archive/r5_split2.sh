#!/bin/bash
# After the descriptor fix: (1) co-resident split (base) vs the T-table claim
# kernel alone (nobs) vs bitsliced waves at issue priority 2 (bsprio), AES-256
# 4 GiB, 2 reps; (2) the claim kernel alone (nobs split) vs the grid T-table
# (ttable) across sizes, ECB-256 and segment encryption.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=${1:-r5_split2}
B="--bits 256 --iters 30 --split-stats"
C="--mode ecb --bytes 4G --impl split $B;--mode cbc-dec --bytes 4G --impl split $B;--mode cfb-dec --bytes 4G --impl split $B"
bash scripts/ab_power.sh $O 2 "$C" base nobs bsprio || exit 1
C=""
for s in 64M 100M 256M 512M 1000M; do C="$C;--mode ecb --bytes $s --impl ttable $B;--mode ecb --bytes $s --impl split $B"; done
for s in 256M 1G 4G; do for g in 4096 512; do
    C="$C;--mode cbc-enc-seg --seg $g --bytes $s --impl ttable $B;--mode cbc-enc-seg --seg $g --bytes $s --impl split $B"
done; done
C="$C;--mode cbc-enc-seg --seg 4096 --bytes 32G --impl ttable --bits 256 --iters 6;--mode cbc-enc-seg --seg 4096 --bytes 32G --impl split --bits 256 --iters 6"
bash scripts/ab_power.sh $O 1 "${C#;}" nobs
