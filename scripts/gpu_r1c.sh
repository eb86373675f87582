#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r1c
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
B="./bin/otbench --bytes 4G --iters 10 --warmup 2 --inplace"
timeout -k 10 300 bash -c "
for bits in 128 256; do
  $B --mode ctr --bits \$bits --impl bitslice || exit 1
  $B --mode ecb --bits \$bits --impl bitslice || exit 1
  $B --mode ctr --bits \$bits --impl ttable || exit 1
done" > $OUT/sweep.jsonl 2>&1 || exit 1
cat $OUT/sweep.jsonl
cd /tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc_bs -o run -- ./bin/otbench --bytes 4G --iters 3 --warmup 1 --mode ctr --impl bitslice --inplace > $OUT/pmc_bs.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $OUT/pmc_bs2 -o run -- ./bin/otbench --bytes 4G --iters 3 --warmup 1 --mode ctr --impl bitslice --inplace > $OUT/pmc_bs2.log 2>&1
echo rc=$?
