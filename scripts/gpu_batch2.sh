#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/batch2
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u benchmarks/batch_ctr.py --no-eager > $OUT/batch.jsonl 2> $OUT/err.log || { tail $OUT/err.log; exit 1; }
timeout -k 10 300 python -u benchmarks/batch_ctr.py --msgs 65536 --size 1504 --keys 1024 --no-eager >> $OUT/batch.jsonl 2>> $OUT/err.log || exit 1
timeout -k 10 300 python -u benchmarks/batch_ctr.py --msgs 262144 --size 4096 --keys 4096 --no-eager >> $OUT/batch.jsonl 2>> $OUT/err.log || exit 1
timeout -k 10 300 python -u benchmarks/batch_ctr.py --msgs 1024 --size 1048576 --keys 64 --no-eager >> $OUT/batch.jsonl 2>> $OUT/err.log || exit 1
python -c "
import json
for l in open('$OUT/batch.jsonl'):
    d=json.loads(l); print(d['msgs'], d['msg_bytes'], d['batch']['gbps'], d['batch_packed']['gbps'], d['batch']['tile_blocks'])
"
