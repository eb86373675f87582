#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/tt2
mkdir -p $OUT
F=$OUT/ab.jsonl
for rep in 1 2; do
for v in default 22x4 22x2; do
  if [ $v = default ]; then unset OTC_TT_VARIANT; else export OTC_TT_VARIANT=$v; fi
  timeout -k 10 120 ./bin/otbench --mode ctr --bits 128 --bytes 4G --inplace --impl ttable --clock --verify | sed "s/}$/, \"variant\": \"$v\"}/" >> $F || exit 1
done
done
unset OTC_TT_VARIANT
cat $F
