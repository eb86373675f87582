#!/bin/bash
# Interleaved A/B of variant libraries (make variant NAME=...) on bitsliced
# CTR at 64 GiB in place, AES-128 and AES-256, REPS rounds, then a --verify
# pass of the last variant at every key size (run on the box):
#   bash scripts/ab_variants.sh REPS name1 name2 ...
# otbench's RUNPATH yields to LD_LIBRARY_PATH, so each variant is loaded from
# variants/NAME/.  Lines "NAME {otbench json}" -> gpurun_out/ab_variants.txt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
reps=$1; shift
O=gpurun_out/ab_variants.txt
mkdir -p gpurun_out
for r in $(seq 1 "$reps"); do for bits in 128 256; do for v in "$@"; do
    line=$(LD_LIBRARY_PATH=variants/$v timeout -k 10 180 ./bin/otbench --mode ctr --bits $bits --bytes 64G \
        --impl bitslice --inplace --iters 10 --warmup 2 --clock) || { echo "FAILED $v $bits"; exit 1; }
    echo "$v $line" | tee -a $O
done; done; done
last=${!#}
for bits in 128 192 256; do
    LD_LIBRARY_PATH=variants/$last timeout -k 10 180 ./bin/otbench --mode ctr --bits $bits --bytes 4G \
        --impl bitslice --iters 2 --verify | sed "s/^/$last verify /" | tee -a $O || exit 1
done
