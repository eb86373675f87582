#!/bin/bash
# RC4 default (auto cap at 10 workgroups per CU) vs forced uncapped: tests, then shapes.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/rc4cap3
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "rc4 or arc4" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for env in "" "0"; do
for shape in "131072 8K" "147456 8K" "163840 8K" "1048576 1K"; do
  set -- $shape
  if [ -z "$env" ]; then unset OTC_RC4_WG_PER_CU; tag=auto; else export OTC_RC4_WG_PER_CU=$env; tag=$env; fi
  timeout -k 10 120 ./bin/otbench --mode rc4 --streams $1 --len $2 --iters 5 --warmup 1 --clock \
    | sed "s/}$/, \"streams\": $1, \"len\": \"$2\", \"wg_cap\": \"$tag\"}/" >> $OUT/rc4.jsonl 2>> $OUT/err.log || exit 1
done
done
python3 -c "
import json
for l in open('$OUT/rc4.jsonl'):
    d=json.loads(l); print(d['wg_cap'], d['streams'], d['len'], d['gbps'], d.get('held_clock_ghz'))"
