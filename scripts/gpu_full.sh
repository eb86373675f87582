#!/bin/bash
# Full validation + kernel sweep + headline bench.  Usage: gpu_full.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/full}
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
B="./bin/otbench --bytes 4G --iters 20 --warmup 3 --clock"
timeout -k 10 900 bash -c "
for bits in 128 256; do
  for impl in ttable bitslice; do
    $B --mode ctr --bits \$bits --impl \$impl --inplace || exit 1
    $B --mode ecb --bits \$bits --impl \$impl || exit 1
  done
  $B --mode ecb-dec --bits \$bits || exit 1
  $B --mode cbc-dec --bits \$bits || exit 1
  $B --mode cbc-enc-seg --bits \$bits --seg 4096 || exit 1
  $B --mode cfb-dec --bits \$bits || exit 1
done
$B --mode xor
$B --mode rc4 --streams 131072 --len 8192 --iters 3
" > $OUT/sweep.jsonl 2>&1 || { tail -5 $OUT/sweep.jsonl; exit 1; }
python - $OUT/sweep.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    try: d=json.loads(l)
    except Exception: continue
    print(f"{d['mode']:12s} {d['bits']} {d['impl']:9s} {d['gbps']:8.1f} GB/s  cpb/cu={d['cycles_per_byte_per_cu']}"
          f"  held={d.get('held_clock_ghz')} GHz cpb/cu@held={d.get('cycles_per_byte_per_cu_held')}")
PY
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1; rc=$?; tail -2 $OUT/bench.log; exit $rc
