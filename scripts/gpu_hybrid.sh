#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/hyb
mkdir -p $OUT
B="./bin/otbench --bytes 4G --iters 10 --warmup 2 --inplace --mode ctr"
timeout -k 10 120 $B --impl hybrid --verify --bytes 256M > $OUT/verify.json 2>&1 || { cat $OUT/verify.json; exit 1; }
cat $OUT/verify.json
timeout -k 10 600 bash -c "
for bits in 128 256; do
  $B --bits \$bits --impl ttable | sed 's/}/, \"variant\": \"tt-1024x4\"}/' || exit 1
  OTC_TT_VARIANT=768x4 $B --bits \$bits --impl ttable | sed 's/}/, \"variant\": \"tt-768x4\"}/' || exit 1
  OTC_TT_VARIANT=768x2 $B --bits \$bits --impl ttable | sed 's/}/, \"variant\": \"tt-768x2\"}/' || exit 1
  for f in 0.5 0.6 0.7 0.8; do
    OTC_HYBRID_TT=\$f $B --bits \$bits --impl hybrid | sed \"s/}/, \\\"variant\\\": \\\"hyb-\$f\\\"}/\" || exit 1
  done
done" > $OUT/sweep.jsonl 2>&1; rc=$?; cat $OUT/sweep.jsonl; exit $rc
