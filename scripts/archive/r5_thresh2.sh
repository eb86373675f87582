#!/bin/bash
# Size thresholds after integer-addressed dynamic LDS: grid T-table (ttable),
# claim kernel alone (nobs split), co-resident split (base split).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=${1:-r5_thresh2}
B="--iters 20 --split-stats"
C=""
for cfg in "ecb --bits 256 --bytes 256M" "ecb --bits 256 --bytes 512M" "ecb --bits 256 --bytes 2G" \
           "cbc-dec --bits 256 --bytes 256M" "cbc-dec --bits 256 --bytes 512M" "cbc-dec --bits 256 --bytes 2G" \
           "ecb --bits 128 --bytes 1G" "ecb --bits 128 --bytes 4G" "cbc-dec --bits 128 --bytes 1G" \
           "cbc-enc-seg --bits 256 --seg 4096 --bytes 256M" "cbc-enc-seg --bits 256 --seg 4096 --bytes 1G" "cbc-enc-seg --bits 256 --seg 4096 --bytes 2G" \
           "cbc-enc-seg --bits 256 --seg 512 --bytes 1G" "cbc-enc-seg --bits 128 --seg 4096 --bytes 4G" "cfb-enc-seg --bits 256 --seg 4096 --bytes 4G"; do
    C="$C;--mode $cfg --impl ttable $B;--mode $cfg --impl split $B"
done
bash scripts/ab_power.sh $O 1 "${C#;}" base nobs
