#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/cfg45
mkdir -p $OUT
timeout -k 10 300 ./bin/otbench --mode ctr --bytes 8G --e2e --chunk 64M --warmup 1 > $OUT/e2e.jsonl 2>&1 &&
timeout -k 10 300 ./bin/otbench --mode ctr --bytes 8G --e2e --chunk 256M --warmup 1 >> $OUT/e2e.jsonl 2>&1 &&
timeout -k 10 300 ./bin/otbench --mode ctr --bytes 8G --e2e --chunk 16M --warmup 1 >> $OUT/e2e.jsonl 2>&1 &&
timeout -k 10 300 ./bin/otbench --mode ctr --bytes 8G --e2e --chunk 64M --warmup 1 --strategy rccl --gpus 1 >> $OUT/e2e.jsonl 2>&1 &&
timeout -k 10 600 python benchmarks/stream_ctr.py --total-gib 64 --window-gib 4 > $OUT/stream_ctr.log 2>&1 &&
timeout -k 10 600 python benchmarks/cbc_scatter.py --gib-per-gpu 16 > $OUT/cbc_scatter.log 2>&1
rc=$?; cat $OUT/e2e.jsonl; tail -2 $OUT/stream_ctr.log $OUT/cbc_scatter.log; exit $rc
