#!/bin/bash
# Final-build kernel sweep (4 GiB, resident), one JSON line per config.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/sweep_final
mkdir -p $OUT
F=$OUT/otbench_sweep.jsonl
run() { timeout -k 10 120 ./bin/otbench "$@" --clock >> $F 2>> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }; }
for bits in 128 192 256; do
  run --mode ctr --bits $bits --bytes 4G --inplace --impl ttable
  run --mode ctr --bits $bits --bytes 4G --inplace --impl bitslice
  run --mode ecb --bits $bits --bytes 4G --impl ttable
  run --mode ecb --bits $bits --bytes 4G --impl bitslice
  run --mode ecb-dec --bits $bits --bytes 4G
  run --mode cbc-dec --bits $bits --bytes 4G
  run --mode cfb-dec --bits $bits --bytes 4G
  run --mode cbc-enc-seg --bits $bits --bytes 4G --seg 4096
done
run --mode xor --bytes 4G
run --mode rc4 --streams 131072 --len 8192 --iters 3
run --mode ecb --bits 128 --bytes 1G --impl ttable --verify
wc -l $F
