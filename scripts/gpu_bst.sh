#!/bin/bash
# Bitsliced with the perm/bit-select transpose: tests + sweep.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/bst
mkdir -p $OUT
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -k "bitslice" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="./bin/otbench --bytes 4G --iters 40 --warmup 10 --inplace --impl bitslice --clock"
timeout -k 10 600 bash -c "
for bits in 128 256; do
  for m in ctr ecb; do
    $B --mode \$m --bits \$bits || exit 1
  done
done
./bin/otbench --bytes 4G --iters 40 --warmup 10 --inplace --impl ttable --clock --mode ctr
" > $OUT/sweep.jsonl 2>&1; rc=$?; cat $OUT/sweep.jsonl; exit $rc
