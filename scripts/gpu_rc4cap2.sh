#!/bin/bash
# RC4 cap A/B at 9 and 10 workgroups per CU (single crowded round), 2 reps.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/rc4cap2
mkdir -p $OUT
for rep in 1 2; do
for cap in 0 6 7; do
for n in 147456 163840; do
  OTC_RC4_WG_PER_CU=$cap timeout -k 10 120 ./bin/otbench --mode rc4 --streams $n --len 8K --iters 5 --warmup 1 --clock \
    | sed "s/}$/, \"streams\": $n, \"len\": \"8K\", \"wg_cap\": $cap}/" >> $OUT/rc4.jsonl 2>> $OUT/err.log || exit 1
done
done
done
python3 -c "
import json
for l in open('$OUT/rc4.jsonl'):
    d=json.loads(l); print(d['wg_cap'], d['streams'], d['gbps'], d.get('held_clock_ghz'))"
