#!/bin/bash
# RC4 i-aligned PRGA (immediate-offset S[i] accesses): RC4 tests, then A/B
# against the generic index arithmetic (OTC_RC4_ALIGNED=0), interleaved.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/rc4align
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "rc4 or xor or arc4" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
for al in 0 1; do
for shape in "131072 8K" "163840 8K" "1048576 1K"; do
  set -- $shape
  OTC_RC4_ALIGNED=$al timeout -k 10 120 ./bin/otbench --mode rc4 --streams $1 --len $2 --iters 5 --warmup 1 --clock \
    | sed "s/}$/, \"streams\": $1, \"len\": \"$2\", \"aligned\": $al}/" >> $OUT/rc4.jsonl 2>> $OUT/err.log || exit 1
done
done
done
cat $OUT/rc4.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['streams'],d['len'],'aligned',d['aligned'],d['gbps'],d.get('held_clock_ghz'))"
