#!/bin/bash
# Pipelined RC4 PRGA: correctness (every stream vs the oracle) + A/B vs the plain loop.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/rc4pipe
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "rc4 or xor" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for ab in pipe plain; do
  if [ $ab = plain ]; then export OTC_RC4_PLAIN=1; fi
  for shape in "131072 8K" "163840 8K" "65536 4K" "1048576 1K"; do
    set -- $shape
    timeout -k 10 120 ./bin/otbench --mode rc4 --streams $1 --len $2 --iters 5 --warmup 1 --clock \
      | sed "s/}$/, \"streams\": $1, \"len\": \"$2\", \"prga\": \"$ab\"}/" >> $OUT/rc4.jsonl 2>> $OUT/err.log || exit 1
  done
done
python -c "
import json
for l in open('$OUT/rc4.jsonl'):
    d=json.loads(l); print(d['prga'], d['streams'], d['len'], d['ms'], d['gbps'], d.get('held_clock_ghz'))
"
