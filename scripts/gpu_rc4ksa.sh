#!/bin/bash
# RC4 KSA for 16-byte keys (register key, i-aligned immediate offsets) vs the
# generic KSA (OTC_RC4_KSA16=0): RC4 tests, then 3 shapes x 2 reps.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/rc4ksa
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "rc4 or arc4" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
for k in 0 1; do
for shape in "131072 8K" "1048576 1K" "1048576 256"; do
  set -- $shape
  OTC_RC4_KSA16=$k timeout -k 10 120 ./bin/otbench --mode rc4 --streams $1 --len $2 --iters 5 --warmup 1 --clock \
    | sed "s/}$/, \"streams\": $1, \"len\": \"$2\", \"ksa16\": $k}/" >> $OUT/rc4.jsonl 2>> $OUT/err.log || exit 1
done
done
done
python3 -c "
import json
for l in open('$OUT/rc4.jsonl'):
    d=json.loads(l); print(d['ksa16'], d['streams'], d['len'], d['gbps'], d.get('held_clock_ghz'))"
