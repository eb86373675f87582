#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/eng
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest.log 2>&1; rc=$?; tail -30 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 ./bin/otbench --mode ctr --bytes 8G --e2e --chunk 256M --warmup 1 > $OUT/e2e.jsonl 2>&1 &&
timeout -k 10 300 ./bin/otbench --mode ctr --bytes 8G --e2e --chunk 64M --warmup 1 >> $OUT/e2e.jsonl 2>&1 &&
timeout -k 10 300 ./bin/otbench --mode ctr --bytes 8G --e2e --chunk 1G --warmup 1 >> $OUT/e2e.jsonl 2>&1 &&
timeout -k 10 300 ./bin/aes_ecb_e > $OUT/aes_ecb_e.txt 2>&1 &&
timeout -k 10 300 ./bin/aes_ecb_e --kernel-only --bits 128 >> $OUT/aes_ecb_e.txt 2>&1 &&
timeout -k 10 120 ./bin/aes_ecb_d 000102030405060708090a0b0c0d0e0f 69c4e0d86a7b0430d8cdb78070b4c55a > $OUT/aes_ecb_d.txt 2>&1 &&
timeout -k 10 600 ./bin/aes_test --suite aesni-ctr,hip-ecb,hip-ctr,hip-cbc --threads 1 --sizes 1048576,104857600,1048576000 > $OUT/aes_test.txt 2>&1 &&
timeout -k 10 600 ./bin/test --device gpu --threads 1 --noselftest > $OUT/rc4_gpu.txt 2>&1
echo rc=$?
cat $OUT/e2e.jsonl $OUT/aes_ecb_e.txt $OUT/aes_ecb_d.txt $OUT/aes_test.txt
