#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r1j
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "rc4 or xor" -x -v --timeout 120 --timeout-method thread > $OUT/pytest_rc4.log 2>&1 || { tail -30 $OUT/pytest_rc4.log; exit 1; }
tail -2 $OUT/pytest_rc4.log
timeout -k 10 120 ./bin/otbench --mode rc4 --streams 131072 --len 8192 --iters 3 --clock > $OUT/rc4.jsonl 2>&1 || { cat $OUT/rc4.jsonl; exit 1; }
timeout -k 10 120 ./bin/otbench --mode rc4 --streams 20480 --len 65536 --iters 3 --clock >> $OUT/rc4.jsonl 2>&1 || exit 1
cat $OUT/rc4.jsonl
