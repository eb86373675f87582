#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r1d
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py -x -q -k "ctr" > $OUT/pytest_ctr.log 2>&1; rc=$?; tail -3 $OUT/pytest_ctr.log; [ $rc -eq 0 ] || exit $rc
B="./bin/otbench --bytes 4G --iters 10 --warmup 2 --inplace --mode ctr --impl ttable"
timeout -k 10 300 bash -c "
for bits in 128 256; do
  OTC_TT_NOCACHE=1 $B --bits \$bits | sed 's/}/, \"variant\": \"nocache\"}/' || exit 1
  for v in 1024x2 512x2 1024x4 1024x1; do
    OTC_TT_VARIANT=\$v $B --bits \$bits | sed \"s/}/, \\\"variant\\\": \\\"cached-\$v\\\"}/\" || exit 1
  done
done" > $OUT/sweep.jsonl 2>&1; rc=$?; cat $OUT/sweep.jsonl; exit $rc
