#!/bin/bash
# RC4 many-stream throughput vs streams per CU (64 streams = one 16 KiB
# workgroup): 4..10 workgroups per CU on 256 CUs, 8 KiB per stream.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/rc4occ
mkdir -p $OUT
for wg in 4 6 8 9 10 11 12; do
  n=$((wg * 256 * 64))
  timeout -k 10 120 ./bin/otbench --mode rc4 --streams $n --len 8K --iters 5 --warmup 1 --clock \
    | sed "s/}$/, \"streams\": $n, \"wg_per_cu\": $wg}/" >> $OUT/rc4.jsonl 2>> $OUT/err.log || exit 1
done
python3 -c "
import json
for l in open('$OUT/rc4.jsonl'):
    d=json.loads(l); print(d['wg_per_cu'], d['streams'], d['gbps'], d.get('held_clock_ghz'))"
