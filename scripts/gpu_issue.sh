#!/bin/bash
# A/B: issue-all-lookups-first round structure vs the interleaved one.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/issue
mkdir -p $OUT
for v in 1024x4 1024x2 2x4; do
  OTC_TT_VARIANT=$v timeout -k 10 120 ./bin/otbench --mode ctr --bytes 64M --iters 3 --verify --impl ttable > $OUT/verify_$v.json 2>&1 || { cat $OUT/verify_$v.json; exit 1; }
  grep -q '"verified": true' $OUT/verify_$v.json || { echo "VERIFY FAIL $v"; cat $OUT/verify_$v.json; exit 1; }
done
for m in ecb ecb-dec cbc-dec; do
  timeout -k 10 120 ./bin/otbench --mode $m --bytes 64M --iters 3 --verify --impl ttable > $OUT/verify_$m.json 2>&1 || { cat $OUT/verify_$m.json; exit 1; }
  grep -q '"verified": true' $OUT/verify_$m.json || { echo "VERIFY FAIL $m"; cat $OUT/verify_$m.json; exit 1; }
done
B="./bin/otbench --bytes 4G --iters 10 --warmup 2 --inplace --impl ttable"
timeout -k 10 600 bash -c "
for bits in 128 256; do
  for v in 1024x4 1024x2 2x4; do
    OTC_TT_VARIANT=\$v $B --mode ctr --bits \$bits | sed \"s/}/, \\\"variant\\\": \\\"\$v\\\"}/\" || exit 1
  done
  $B --mode ecb --bits \$bits || exit 1
done" > $OUT/sweep.jsonl 2>&1; rc=$?; cat $OUT/sweep.jsonl; exit $rc
