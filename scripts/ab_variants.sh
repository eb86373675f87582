#!/bin/bash
# Interleaved A/B of variant libraries (make variant NAME=...) on bitsliced
# CTR at 64 GiB in place, AES-128 and AES-256, REPS rounds, then a --verify
# pass of the last variant at every key size (run on the box):
#   bash scripts/ab_variants.sh REPS name1 name2 ...
# env: AB_MODES (default "ctr"), AB_BITS ("128 256"), AB_IMPL (bitslice),
# AB_BYTES (64G); chained decrypts (cbc-dec, cfb-dec) run out of place
# otbench's RUNPATH yields to LD_LIBRARY_PATH, so each variant is loaded from
# variants/NAME/.  Lines "NAME {otbench json}" -> gpurun_out/ab_variants.txt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
reps=$1; shift
O=gpurun_out/ab_variants.txt
mkdir -p gpurun_out
for r in $(seq 1 "$reps"); do for m in ${AB_MODES:-ctr}; do for bits in ${AB_BITS:-128 256}; do for v in "$@"; do
    ip=--inplace
    case $m in cbc-dec|cfb-dec) ip= ;; esac
    line=$(LD_LIBRARY_PATH=variants/$v timeout -k 10 180 ./bin/otbench --mode $m --bits $bits --bytes ${AB_BYTES:-64G} \
        --impl ${AB_IMPL:-bitslice} $ip --iters 10 --warmup 2 --clock) || { echo "FAILED $v $m $bits"; exit 1; }
    echo "$v $line" | tee -a $O
done; done; done; done
last=${!#}
for m in ${AB_MODES:-ctr}; do for bits in 128 192 256; do
    LD_LIBRARY_PATH=variants/$last timeout -k 10 180 ./bin/otbench --mode $m --bits $bits --bytes 4G \
        --impl ${AB_IMPL:-bitslice} --iters 2 --verify | sed "s/^/$last verify /" | tee -a $O || exit 1
done; done
