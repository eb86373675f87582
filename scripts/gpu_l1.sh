#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/l1
mkdir -p $OUT
for v in 1x4 1x2; do
OTC_TT_VARIANT=$v timeout -k 10 120 ./bin/otbench --mode ctr --bytes 256M --iters 2 --impl ttable --verify > $OUT/v_$v.json 2>&1 && grep -q '"verified": true' $OUT/v_$v.json || { cat $OUT/v_$v.json; exit 1; }
done
B="./bin/otbench --bytes 4G --iters 10 --warmup 2 --inplace --mode ctr --impl ttable"
timeout -k 10 600 bash -c "
for bits in 128 256; do
  for v in 1024x4 1x4 1x2; do
    OTC_TT_VARIANT=\$v $B --bits \$bits | sed \"s/}/, \\\"variant\\\": \\\"\$v\\\"}/\" || exit 1
  done
done" > $OUT/sweep.jsonl 2>&1; rc=$?; cut -c1-60,100-130,200-300 $OUT/sweep.jsonl; exit $rc
