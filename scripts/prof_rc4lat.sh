#!/bin/bash
# RC4 PRGA: LDS latency / queueing counters for the generic (0) and default
# read-ahead (2) loops.  Average LDS latency = SQ_INST_LEVEL_LDS / SQ_INSTS_LDS.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/profrc4lat
mkdir -p $OUT
C="SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
for al in 0 2; do
  OTC_RC4_ALIGNED=$al timeout -s KILL 90 rocprofv3 --pmc $C -d $OUT/al$al -o rc4 -- ./bin/otbench --mode rc4 --streams 131072 --len 8K --iters 4 --warmup 1 > $OUT/al$al.log 2>&1 || { tail -20 $OUT/al$al.log; exit 1; }
done
ls $OUT
