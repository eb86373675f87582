#!/bin/bash
# T-table vs bitsliced crossover (the impl="auto" thresholds), run on the box:
#   bash scripts/xover.sh "128 256" "256M 1G 2G 4G 8G" [MODE] [OUT]
# MODE: an otbench --mode with both kernels (ctr, default; ecb).  2 reps,
# interleaved, in place, JSON lines appended to gpurun_out/OUT (xover.jsonl).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mode=${3:-ctr}
out=gpurun_out/${4:-xover.jsonl}
mkdir -p gpurun_out
for bits in $1; do for b in $2; do for rep in 1 2; do for i in ttable bitslice; do
    timeout -k 10 180 ./bin/otbench --mode "$mode" --bits "$bits" --bytes "$b" --impl $i --iters 20 --inplace \
        >> "$out" || exit 1
done; done; done; done
cat "$out"
