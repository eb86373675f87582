#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r1i
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_batch.log 2>&1 || { tail -30 $OUT/pytest_batch.log; exit 1; }
tail -2 $OUT/pytest_batch.log
timeout -k 10 300 python -u benchmarks/batch_ctr.py --no-eager > $OUT/batch.json 2> $OUT/err.log || { tail $OUT/err.log; exit 1; }
timeout -k 10 300 python -u benchmarks/batch_ctr.py --msgs 65536 --size 1504 --keys 1024 --no-eager >> $OUT/batch.json 2>> $OUT/err.log || exit 1
timeout -k 10 300 python -u benchmarks/batch_ctr.py --msgs 262144 --size 4096 --keys 4096 --no-eager >> $OUT/batch.json 2>> $OUT/err.log || exit 1
cat $OUT/batch.json
