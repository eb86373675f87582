#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/small
mkdir -p $OUT
for b in 64K 1M 10M 100M 1000M; do
  for m in ctr ecb; do
    timeout -k 10 120 ./bin/otbench --mode $m --bits 128 --bytes $b --iters 50 --warmup 5 --impl ttable >> $OUT/small.jsonl 2>> $OUT/err.log || exit 1
  done
done
python -c "
import json
for l in open('$OUT/small.jsonl'):
    d=json.loads(l); print(d['mode'], d['bytes'], d['ms'], d['gbps'])
"
