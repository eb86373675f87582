#!/bin/bash
# CTR split (tables built before the fork) vs bitsliced alone by size.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
C=""
for cfg in "--bits 128 --bytes 8G --inplace --iters 20" "--bits 128 --bytes 16G --inplace --iters 15" "--bits 128 --bytes 32G --inplace --iters 10" \
           "--bits 256 --bytes 1G --iters 20" "--bits 256 --bytes 2G --iters 20" "--bits 192 --bytes 4G --iters 20" "--bits 192 --bytes 64G --inplace --iters 10"; do
    for i in bitslice split; do C="$C;--mode ctr $cfg --impl $i --split-stats"; done
done
bash scripts/ab_power.sh ${1:-r5_ctr_thresh} 2 "${C#;}" base
