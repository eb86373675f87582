#!/bin/bash
# Hybrid CTR sweep: T-table variant (co-residency) x T-table share.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/hybrid2
mkdir -p $OUT
for v in 1024x2 512x4; do
  OTC_TT_VARIANT=$v OTC_HYBRID_TT=0.6 timeout -k 10 120 ./bin/otbench --mode ctr --bytes 64M --iters 3 --verify --impl hybrid > $OUT/verify_$v.json 2>&1 || { cat $OUT/verify_$v.json; exit 1; }
  grep -q '"verified": true' $OUT/verify_$v.json || { echo "VERIFY FAIL $v"; cat $OUT/verify_$v.json; exit 1; }
done
B="./bin/otbench --bytes 4G --iters 40 --warmup 10 --inplace --mode ctr --bits 128"
timeout -k 10 900 bash -c "
$B --impl ttable | sed 's/}/, \"tag\": \"tt\"}/' || exit 1
$B --impl bitslice | sed 's/}/, \"tag\": \"bs\"}/' || exit 1
for v in 1024x2 512x4; do
  OTC_TT_VARIANT=\$v $B --impl ttable | sed \"s/}/, \\\"tag\\\": \\\"tt \$v\\\"}/\" || exit 1
  for f in 0.5 0.6 0.7 0.8; do
    OTC_TT_VARIANT=\$v OTC_HYBRID_TT=\$f $B --impl hybrid | sed \"s/}/, \\\"tag\\\": \\\"hy \$v \$f\\\"}/\" || exit 1
  done
done
$B --impl ttable | sed 's/}/, \"tag\": \"tt\"}/' || exit 1
" > $OUT/sweep.jsonl 2>&1; rc=$?; cat $OUT/sweep.jsonl; exit $rc
