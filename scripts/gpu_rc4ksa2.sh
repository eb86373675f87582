#!/bin/bash
# Register KSA for key lengths dividing 32: RC4 tests (incl. 32/8/2-byte keys),
# then 16-byte-key shapes for regression.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/rc4ksa2
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "rc4 or arc4" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for shape in "131072 8K" "1048576 1K" "1048576 256"; do
  set -- $shape
  timeout -k 10 120 ./bin/otbench --mode rc4 --streams $1 --len $2 --iters 5 --warmup 1 --clock \
    | sed "s/}$/, \"streams\": $1, \"len\": \"$2\"}/" >> $OUT/rc4.jsonl 2>> $OUT/err.log || exit 1
done
python3 -c "
import json
for l in open('$OUT/rc4.jsonl'):
    d=json.loads(l); print(d['streams'], d['len'], d['gbps'], d.get('held_clock_ghz'))"
