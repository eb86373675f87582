#!/bin/bash
# LDS pipe counters for the cached 4-table CTR kernel (issue-all and interleaved).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/proflds2
mkdir -p $OUT
B="./bin/otbench --bytes 4G --iters 3 --warmup 1 --inplace --mode ctr --impl ttable"
run() {  # name variant counters...
  local n=$1 v=$2; shift 2
  OTC_TT_VARIANT=$v timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$n -o run -- $B > $OUT/$n.log 2>&1
}
OTC_TT_VARIANT=1024x4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- $B > $OUT/kt.log 2>&1 &&
run a1 1024x4 GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INST_LEVEL_LDS SQ_WAVES SQ_BUSY_CYCLES &&
run a2 1024x4 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU &&
run b1 2x4 GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INST_LEVEL_LDS SQ_WAVES SQ_BUSY_CYCLES &&
run b2 2x4 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
rc=$?
echo rc=$rc; find $OUT -name '*.csv' | head -20
exit $rc
