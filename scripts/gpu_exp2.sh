#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/exp2
mkdir -p $OUT
B="./bin/otbench --bytes 4G --iters 10 --warmup 2 --inplace --mode ctr"
OTC_BS_CTR_CACHE=1 timeout -k 10 120 $B --impl bitslice --verify --bytes 256M --inplace > /dev/null 2>&1
timeout -k 10 120 ./bin/otbench --mode ctr --bytes 256M --iters 2 --impl bitslice --verify > $OUT/v1.json 2>&1 && grep -q '"verified": true' $OUT/v1.json || { cat $OUT/v1.json; exit 1; }
OTC_BS_CTR_CACHE=1 timeout -k 10 120 ./bin/otbench --mode ctr --bytes 256M --iters 2 --impl bitslice --verify > $OUT/v2.json 2>&1 && grep -q '"verified": true' $OUT/v2.json || { cat $OUT/v2.json; exit 1; }
OTC_TT_VARIANT=1024x2 timeout -k 10 120 ./bin/otbench --mode ctr --bytes 256M --iters 2 --impl hybrid --verify > $OUT/v3.json 2>&1 && grep -q '"verified": true' $OUT/v3.json || { cat $OUT/v3.json; exit 1; }
timeout -k 10 600 bash -c "
for bits in 128 256; do
  $B --bits \$bits --impl bitslice | sed 's/}/, \"variant\": \"bs-nocache\"}/' || exit 1
  OTC_BS_CTR_CACHE=1 $B --bits \$bits --impl bitslice | sed 's/}/, \"variant\": \"bs-cache\"}/' || exit 1
  $B --bits \$bits --impl ttable | sed 's/}/, \"variant\": \"tt\"}/' || exit 1
  for f in 0.7 0.8 0.9; do
    OTC_TT_VARIANT=1024x2 OTC_HYBRID_TT=\$f $B --bits \$bits --impl hybrid | sed \"s/}/, \\\"variant\\\": \\\"hyb-b2-\$f\\\"}/\" || exit 1
  done
done" > $OUT/sweep.jsonl 2>&1; rc=$?; cat $OUT/sweep.jsonl | cut -c1-60,100-130,200-300; exit $rc
