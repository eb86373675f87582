#!/bin/bash
# Where the co-resident split (base, impl split) and the T-table claim kernel
# alone (nobs, impl split) beat the grid T-table (impl ttable), by size.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=${1:-r5_thresh}
B="--iters 20 --split-stats"
C=""
for m in ecb cbc-dec cfb-dec; do for s in 1G 2G 4G 16G; do
    C="$C;--mode $m --bits 256 --bytes $s --impl ttable $B;--mode $m --bits 256 --bytes $s --impl split $B"
done; done
for m in ecb cbc-dec; do C="$C;--mode $m --bits 128 --bytes 4G --impl ttable $B;--mode $m --bits 128 --bytes 4G --impl split $B"; done
bash scripts/ab_power.sh $O 1 "${C#;}" base || exit 1
C=""
for s in 2G 8G; do for g in 4096 512; do
    C="$C;--mode cbc-enc-seg --bits 256 --seg $g --bytes $s --impl ttable $B;--mode cbc-enc-seg --bits 256 --seg $g --bytes $s --impl split $B"
done; done
C="$C;--mode cfb-enc-seg --bits 256 --seg 4096 --bytes 4G --impl ttable $B;--mode cfb-enc-seg --bits 256 --seg 4096 --bytes 4G --impl split $B"
C="$C;--mode cbc-enc-seg --bits 128 --seg 4096 --bytes 4G --impl ttable $B;--mode cbc-enc-seg --bits 128 --seg 4096 --bytes 4G --impl split $B"
bash scripts/ab_power.sh $O 1 "${C#;}" nobs
