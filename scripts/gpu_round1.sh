#!/bin/bash
# First GPU validation pass: correctness smoke, pytest -m gpu, kernel sweeps.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r1
mkdir -p $OUT
rocm-smi --showproductname > $OUT/smi.txt 2>&1 || true
run() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name" ; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -3 $OUT/$name.log
  return $rc
}
run otb_ctr_tt 120 ./bin/otbench --mode ctr --bytes 64M --iters 5 --verify --impl ttable &&
run otb_ctr_bs 120 ./bin/otbench --mode ctr --bytes 64M --iters 5 --verify --impl bitslice &&
run otb_ecb_tt 120 ./bin/otbench --mode ecb --bytes 64M --iters 5 --verify --impl ttable &&
run otb_ecbdec 120 ./bin/otbench --mode ecb-dec --bytes 64M --iters 5 --verify &&
run otb_cbcdec 120 ./bin/otbench --mode cbc-dec --bytes 64M --iters 5 --verify &&
run pytest_gpu 900 python -m pytest tests -m gpu -x -q &&
run sweep 600 bash -c '
for b in 128 256; do for impl in ttable bitslice; do
  ./bin/otbench --mode ctr --bits $b --bytes 4G --iters 10 --impl $impl --inplace || exit 1
  ./bin/otbench --mode ecb --bits $b --bytes 4G --iters 10 --impl $impl || exit 1
done
  ./bin/otbench --mode ecb-dec --bits $b --bytes 4G --iters 10 || exit 1
  ./bin/otbench --mode cbc-dec --bits $b --bytes 4G --iters 10 || exit 1
  ./bin/otbench --mode cbc-enc-seg --bits $b --bytes 4G --seg 4096 --iters 5 || exit 1
  ./bin/otbench --mode cfb-dec --bits $b --bytes 4G --iters 5 || exit 1
done
./bin/otbench --mode xor --bytes 4G --iters 10
./bin/otbench --mode rc4 --streams 131072 --len 8192 --iters 3
' &&
run bench_8g 300 python bench.py --gib 8 --steps 10 --warmup 2 &&
run bench_default 600 python bench.py
echo ALLDONE
