#!/bin/bash
# Batch tile sizes + non-temporal A/B on the headline CTR kernel.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r1g
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_batch.log 2>&1 || { tail -30 $OUT/pytest_batch.log; exit 1; }
tail -2 $OUT/pytest_batch.log
for t in 64 128 256; do
  timeout -k 10 300 python -u benchmarks/batch_ctr.py --msgs 65536 --size 1504 --keys 1024 --no-eager --tile $t >> $OUT/batch_tiles.jsonl 2>> $OUT/err.log || exit 1
  timeout -k 10 300 python -u benchmarks/batch_ctr.py --msgs 16384 --size 4096 --keys 256 --no-eager --tile $t >> $OUT/batch_tiles.jsonl 2>> $OUT/err.log || exit 1
done
cat $OUT/batch_tiles.jsonl
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --no-aes256 --no-bitslice >> $OUT/nt_ab.jsonl 2>> $OUT/err.log || exit 1
  OTC_TT_NT=1 timeout -k 10 300 python -u bench.py --steps 10 --no-aes256 --no-bitslice >> $OUT/nt_ab.jsonl 2>> $OUT/err.log || exit 1
done
grep -o '"value": [0-9.]*\|held_clock_ghz": [0-9.]*' $OUT/nt_ab.jsonl
