#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/tbl4
mkdir -p $OUT
for v in -1024x4 -1024x2 -512x4; do
  OTC_TT_VARIANT=$v timeout -k 10 120 ./bin/otbench --mode ctr --bytes 64M --iters 3 --verify --impl ttable > $OUT/verify_$v.json 2>&1 || { cat $OUT/verify_$v.json; exit 1; }
  grep -q '"verified": true' $OUT/verify_$v.json || { echo "VERIFY FAIL $v"; cat $OUT/verify_$v.json; exit 1; }
done
B="./bin/otbench --bytes 4G --iters 10 --warmup 2 --inplace --mode ctr --impl ttable"
timeout -k 10 600 bash -c "
for bits in 128 256; do
  for v in 1024x4 -1024x4 -1024x2 -512x4; do
    OTC_TT_VARIANT=\$v $B --bits \$bits | sed \"s/}/, \\\"variant\\\": \\\"\$v\\\"}/\" || exit 1
  done
done" > $OUT/sweep.jsonl 2>&1; rc=$?; cat $OUT/sweep.jsonl; exit $rc
