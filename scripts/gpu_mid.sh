#!/bin/bash
# Mid-size launch shape (1024-block steps when they balance the CUs better):
# full GPU tests incl. the hypothesis fuzz tests, then an A/B over sizes.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/mid
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for ab in mid bulk; do
  if [ $ab = bulk ]; then export OTC_TT_NOMID=1; fi
  for b in 5M 10M 24M 100M 300M 1G; do
    for m in ctr ecb ecb-dec; do
      timeout -k 10 120 ./bin/otbench --mode $m --bits 128 --bytes $b --iters 30 --warmup 3 --verify | sed "s/}$/, \"shape\": \"$ab\"}/" >> $OUT/mid.jsonl 2>> $OUT/err.log || exit 1
    done
  done
done
python -c "
import json
for l in open('$OUT/mid.jsonl'):
    d=json.loads(l); print(d['shape'], d['mode'], d['bytes'], d['ms'], d['gbps'], d['verified'])
"
