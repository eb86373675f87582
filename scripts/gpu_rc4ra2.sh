#!/bin/bash
# RC4 read-ahead in the KSA and drop loops too (default, AL=2) vs without
# (OTC_RC4_ALIGNED=1): RC4 tests, then 1M x 1 KiB at keylen 16/32, drop 0/768, 2 reps.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/rc4ra2
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "rc4 or arc4" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
for al in 1 2; do
for kl in 16 32; do
for drop in 0 768; do
  OTC_RC4_ALIGNED=$al timeout -k 10 120 ./bin/otbench --mode rc4 --streams 1048576 --len 1K --keylen $kl --drop $drop --iters 5 --warmup 1 \
    | sed "s/}$/, \"keylen\": $kl, \"drop\": $drop, \"variant\": $al}/" >> $OUT/rc4.jsonl 2>> $OUT/err.log || exit 1
done
done
done
done
python3 -c "
import json
for l in open('$OUT/rc4.jsonl'):
    d=json.loads(l); print('variant',d['variant'],'keylen',d['keylen'],'drop',d['drop'], d['gbps'])"
