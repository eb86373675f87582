#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r1b
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
B="./bin/otbench --bytes 4G --iters 10 --warmup 2 --inplace"
timeout -k 10 600 bash -c "
for bits in 128 256; do
  $B --mode ctr --bits \$bits --impl bitslice || exit 1
  $B --mode ecb --bits \$bits --impl bitslice || exit 1
  for v in 512x2 1024x2 512x4 1024x4 256x4 512x1 1024x1; do
    OTC_TT_VARIANT=\$v $B --mode ctr --bits \$bits --impl ttable | sed \"s/}/, \\\"variant\\\": \\\"\$v\\\"}/\" || exit 1
  done
done" > $OUT/sweep.jsonl 2>&1; rc=$?; cat $OUT/sweep.jsonl; exit $rc
