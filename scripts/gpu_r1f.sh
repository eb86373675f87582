#!/bin/bash
# Batched CTR + graph capture tests, full GPU suite, serving benchmark, CBC scatter pipeline (1 GPU).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r1f
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_batch.log 2>&1 || { tail -30 $OUT/pytest_batch.log; exit 1; }
tail -2 $OUT/pytest_batch.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u benchmarks/batch_ctr.py > $OUT/batch_ctr.json 2> $OUT/batch_ctr.err || { tail -20 $OUT/batch_ctr.err; exit 1; }
cat $OUT/batch_ctr.json
timeout -k 10 300 python -u benchmarks/batch_ctr.py --msgs 65536 --size 1504 --keys 1024 --no-eager > $OUT/batch_ctr_small.json 2>> $OUT/batch_ctr.err || exit 1
cat $OUT/batch_ctr_small.json
timeout -k 10 300 python -u benchmarks/cbc_scatter.py --gib-per-gpu 16 > $OUT/cbc_scatter.json 2>&1 || { tail -20 $OUT/cbc_scatter.json; exit 1; }
cat $OUT/cbc_scatter.json
