#!/bin/bash
# RC4 PRGA A/B: 2 (read-ahead, conflict-free layout) vs 3 (same loop, byte-interleaved layout).
# RC4 tests under variant 3 and the default first.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/rc4bl
mkdir -p $OUT
OTC_RC4_ALIGNED=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "rc4 or arc4" -x -q --timeout 120 --timeout-method thread > $OUT/pytest2.log 2>&1 || { tail -30 $OUT/pytest2.log; exit 1; }
tail -1 $OUT/pytest2.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "rc4 or arc4" -x -q --timeout 120 --timeout-method thread > $OUT/pytest1.log 2>&1 || { tail -30 $OUT/pytest1.log; exit 1; }
tail -1 $OUT/pytest1.log
for rep in 1 2; do
for al in 2 3; do
for shape in "131072 8K" "1048576 1K"; do
  set -- $shape
  OTC_RC4_ALIGNED=$al timeout -k 10 120 ./bin/otbench --mode rc4 --streams $1 --len $2 --iters 5 --warmup 1 --clock \
    | sed "s/}$/, \"streams\": $1, \"len\": \"$2\", \"variant\": $al}/" >> $OUT/rc4.jsonl 2>> $OUT/err.log || exit 1
done
done
done
cat $OUT/rc4.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['streams'],d['len'],'variant',d['variant'],d['gbps'],d.get('held_clock_ghz'))"
