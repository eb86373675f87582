#!/bin/bash
# After integer-addressed dynamic LDS in the T-table claim kernels: grid
# T-table (ttable) vs claim kernel alone (nobs split) vs co-resident split
# (base split), AES-256, with power.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=${1:-r5_remeasure}
B="--bits 256 --iters 20 --split-stats"
C=""
for cfg in "ecb --bytes 4G" "ecb --bytes 64G --inplace" "cbc-dec --bytes 16G" "cfb-dec --bytes 16G" "ecb --bytes 1G" "cbc-dec --bytes 1G" \
           "cbc-enc-seg --seg 4096 --bytes 4G" "cbc-enc-seg --seg 512 --bytes 4G" "cbc-enc-seg --seg 4096 --bytes 32G"; do
    C="$C;--mode $cfg --impl ttable $B;--mode $cfg --impl split $B"
done
bash scripts/ab_power.sh $O 1 "${C#;}" base nobs
