#!/bin/bash
# otbench RC4 with --keylen/--drop: 1M x 1 KiB, key lengths 5/16/32, drop 0/768,
# default loops vs generic (OTC_RC4_ALIGNED=0 OTC_RC4_KSA16=0).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/rc4keylen
mkdir -p $OUT
for kl in 5 16 32; do
for drop in 0 768; do
for gen in 0 1; do
  if [ $gen = 1 ]; then export OTC_RC4_ALIGNED=0 OTC_RC4_KSA16=0; else unset OTC_RC4_ALIGNED OTC_RC4_KSA16; fi
  timeout -k 10 120 ./bin/otbench --mode rc4 --streams 1048576 --len 1K --keylen $kl --drop $drop --iters 5 --warmup 1 \
    | sed "s/}$/, \"keylen\": $kl, \"drop\": $drop, \"generic\": $gen}/" >> $OUT/rc4.jsonl 2>> $OUT/err.log || exit 1
done
done
done
python3 -c "
import json
for l in open('$OUT/rc4.jsonl'):
    d=json.loads(l); print('keylen',d['keylen'],'drop',d['drop'],'generic',d['generic'], d['gbps'])"
