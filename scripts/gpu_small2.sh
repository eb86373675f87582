#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/small2
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for ab in small bulk; do
  if [ $ab = bulk ]; then export OTC_TT_NOSMALL=1; fi
  for b in 64K 256K 1M 4M 10M 100M; do
    for m in ctr ecb ecb-dec; do
      timeout -k 10 120 ./bin/otbench --mode $m --bits 128 --bytes $b --iters 50 --warmup 5 --verify | sed "s/}$/, \"shape\": \"$ab\"}/" >> $OUT/small.jsonl 2>> $OUT/err.log || exit 1
    done
  done
done
python -c "
import json
for l in open('$OUT/small.jsonl'):
    d=json.loads(l); print(d['shape'], d['mode'], d['bytes'], d['ms'], d['gbps'], d['verified'])
"
