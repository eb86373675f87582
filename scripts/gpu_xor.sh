#!/bin/bash
# XOR combiner (device arc4_crypt) A/B: loads per lane per trip x workgroups per CU x nt.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/xor
mkdir -p $OUT
: > $OUT/xor.jsonl
for v in 1,8,0 1,16,0 1,32,0 2,8,0 2,16,0 4,4,0 4,8,0 4,16,0 8,4,0 8,8,0 1,8,1 2,16,1 4,8,1 4,16,1; do
  for b in 1G 4G; do
    OTC_XOR_VARIANT=$v timeout -k 10 60 ./bin/otbench --mode xor --bytes $b --iters 30 --warmup 3 --clock \
      | sed "s/}$/, \"variant\": \"$v\"}/" >> $OUT/xor.jsonl 2>> $OUT/err.log || exit 1
  done
done
python -c "
import json
for l in open('$OUT/xor.jsonl'):
    d=json.loads(l); print(d['variant'], d['bytes']>>20, 'MiB', d['ms'], d['gbps'], d.get('held_clock_ghz'))
"
