#!/bin/bash
# LDS / issue counters of the many-stream RC4 kernel (plain and pipelined PRGA),
# 131072 streams x 8 KiB; one pass per counter set (<= 8 SQ counters).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/profrc4
mkdir -p $OUT
B="./bin/otbench --mode rc4 --streams 131072 --len 8K --iters 3 --warmup 1"
run() {  # name plain(0/1) counters...
  local n=$1 p=$2; shift 2
  if [ $p = 1 ]; then export OTC_RC4_PLAIN=1; else unset OTC_RC4_PLAIN; fi
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$n -o run -- $B > $OUT/$n.log 2>&1
}
C1="GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_WAVES SQ_BUSY_CYCLES"
C2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
C3="SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INST_LEVEL_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- $B > $OUT/kt.log 2>&1 &&
run plain1 1 $C1 && run plain2 1 $C2 && run plain3 1 $C3 &&
run pipe1 0 $C1 && run pipe2 0 $C2 && run pipe3 0 $C3
rc=$?
echo rc=$rc; find $OUT -name '*counter_collection.csv' | head -20
exit $rc
