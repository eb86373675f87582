#!/bin/bash
# CBC-encrypt segments: grouped load/store bursts (OTC_CBC_GROUP = 1 | 4 | 8).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/cbcenc
mkdir -p $OUT
for g in 1 4 8; do
  OTC_CBC_GROUP=$g timeout -k 10 120 ./bin/otbench --mode cbc-enc-seg --bytes 64M --iters 3 --verify > $OUT/verify_$g.json 2>&1 || { cat $OUT/verify_$g.json; exit 1; }
  grep -q '"verified": true' $OUT/verify_$g.json || { echo "VERIFY FAIL $g"; cat $OUT/verify_$g.json; exit 1; }
done
timeout -k 10 120 python -m pytest tests/test_gpu_kernels.py -q -x -k "cbc_segments or single_segment" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
B="./bin/otbench --bytes 4G --iters 20 --warmup 3 --mode cbc-enc-seg"
timeout -k 10 600 bash -c "
for bits in 128 256; do
  for g in 1 4 8 1 4; do
    OTC_CBC_GROUP=\$g $B --bits \$bits | sed \"s/}/, \\\"group\\\": \$g}/\" || exit 1
  done
done" > $OUT/sweep.jsonl 2>&1; rc=$?; cat $OUT/sweep.jsonl; exit $rc
