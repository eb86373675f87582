#!/bin/bash
# rocprofv3: kernel-trace stats + PMC counters for the AES kernels.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=gpurun_out/prof1
mkdir -p $OUT
B="./bin/otbench --bytes 4G --iters 3 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B --mode ctr --impl ttable > $OUT/trace_tt.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_bs -o run -- $B --mode ctr --impl bitslice > $OUT/trace_bs.log 2>&1 &&
for impl in ttable bitslice; do
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/pmc1_$impl -o run -- $B --mode ctr --impl $impl > $OUT/pmc1_$impl.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/pmc2_$impl -o run -- $B --mode ctr --impl $impl > $OUT/pmc2_$impl.log 2>&1 || exit 1
done
echo done
find $OUT -name '*.csv' | head -40
