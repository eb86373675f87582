#!/bin/bash
# Instruction-cache and issue counters: bitsliced CTR (150 KB of code) vs T-table CTR.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/profbs
mkdir -p $OUT
for impl in bitslice ttable; do
  B="./bin/otbench --bytes 4G --iters 3 --warmup 1 --inplace --mode ctr --impl $impl"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$impl -o run -- $B > $OUT/kt_$impl.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES --output-format csv -d $OUT/p1_$impl -o run -- $B > $OUT/p1_$impl.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $OUT/p2_$impl -o run -- $B > $OUT/p2_$impl.log 2>&1 || exit 1
done
echo done
