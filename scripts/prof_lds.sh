#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/proflds
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1
grep -oE '(SQ|SQC|TA|TD|TCP|TCC|GRBM|SPI)_[A-Z0-9_]+' $OUT/counters_list.txt | sort -u > $OUT/counter_names.txt
B="./bin/otbench --bytes 4G --iters 3 --warmup 1 --inplace --mode ctr --impl ttable"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES --output-format csv -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL --output-format csv -d $OUT/p2 -o run -- $B > $OUT/p2.log 2>&1
echo rc=$?; tail -3 $OUT/p1.log $OUT/p2.log; wc -l $OUT/counter_names.txt
