#!/bin/bash
# A/B: bitsliced CTR plaintext prefetch distance (OTC_BS_PF).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/bspf
mkdir -p $OUT
for pf in 0 4 8; do
  for bits in 128 256; do
    OTC_BS_PF=$pf timeout -k 10 120 ./bin/otbench --mode ctr --bits $bits --bytes 64M --iters 3 --verify --impl bitslice > $OUT/verify_${pf}_$bits.json 2>&1 || { cat $OUT/verify_${pf}_$bits.json; exit 1; }
    grep -q '"verified": true' $OUT/verify_${pf}_$bits.json || { echo "VERIFY FAIL $pf"; cat $OUT/verify_${pf}_$bits.json; exit 1; }
  done
done
B="./bin/otbench --bytes 4G --iters 60 --warmup 10 --inplace --impl bitslice --mode ctr"
timeout -k 10 600 bash -c "
for bits in 128; do
  for pf in 0 8 0 8 4 0 8; do
    OTC_BS_PF=\$pf $B --bits \$bits | sed \"s/}/, \\\"pf\\\": \$pf}/\" || exit 1
  done
done" > $OUT/sweep.jsonl 2>&1; rc=$?; cat $OUT/sweep.jsonl; exit $rc
