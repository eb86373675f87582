#!/bin/bash
# T-table vs bitsliced CTR crossover (the impl="auto" thresholds), run on the box:
#   bash scripts/xover.sh "128 256" "256M 1G 2G 4G 8G"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for bits in $1; do for b in $2; do for rep in 1 2; do for i in ttable bitslice; do
    timeout -k 10 180 ./bin/otbench --mode ctr --bits "$bits" --bytes "$b" --impl $i --iters 20 --inplace \
        >> gpurun_out/xover.jsonl || exit 1
done; done; done; done
cat gpurun_out/xover.jsonl
