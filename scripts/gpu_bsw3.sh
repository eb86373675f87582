#!/bin/bash
# A/B: bitsliced at 3 waves/SIMD with scratch spills (OTC_BS_W3=1) vs default.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/bsw3
mkdir -p $OUT
for m in ctr ecb; do
  OTC_BS_W3=1 timeout -k 10 120 ./bin/otbench --mode $m --bytes 64M --iters 3 --verify --impl bitslice > $OUT/verify_$m.json 2>&1 || { cat $OUT/verify_$m.json; exit 1; }
  grep -q '"verified": true' $OUT/verify_$m.json || { echo "VERIFY FAIL $m"; exit 1; }
done
B="./bin/otbench --bytes 4G --iters 40 --warmup 10 --inplace --impl bitslice --clock"
timeout -k 10 600 bash -c "
for bits in 128 256; do
  for m in ctr ecb; do
    for w in 0 1 0 1; do
      OTC_BS_W3=\$w $B --mode \$m --bits \$bits | sed \"s/}/, \\\"w3\\\": \$w}/\" || exit 1
    done
  done
done" > $OUT/sweep.jsonl 2>&1; rc=$?; cat $OUT/sweep.jsonl; exit $rc
