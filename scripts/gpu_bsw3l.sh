#!/bin/bash
# A/B: 3-waves/SIMD bitsliced CTR with / without the 12-slot LDS prefetch.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/bsw3l
mkdir -p $OUT
for bits in 128 256; do
  OTC_BS_W3=1 timeout -k 10 120 ./bin/otbench --mode ctr --bits $bits --bytes 64M --iters 3 --verify --impl bitslice > $OUT/verify_$bits.json 2>&1 || { cat $OUT/verify_$bits.json; exit 1; }
  grep -q '"verified": true' $OUT/verify_$bits.json || { echo "VERIFY FAIL $bits"; exit 1; }
done
OTC_BS_W3=1 timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -k "bitslice" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="./bin/otbench --bytes 4G --iters 40 --warmup 10 --inplace --impl bitslice --clock --mode ctr"
timeout -k 10 600 bash -c "
for bits in 128 256; do
  for l in 0 1 0 1; do
    OTC_BS_W3=1 OTC_BS_LDS=\$l $B --bits \$bits | sed \"s/}/, \\\"lds\\\": \$l}/\" || exit 1
  done
done" > $OUT/sweep.jsonl 2>&1; rc=$?; cat $OUT/sweep.jsonl; exit $rc
