#!/bin/bash
# VALU counters of the final bitsliced CTR kernel (3 waves/SIMD build) and of
# the batched T-table kernel, one pass each (<= 8 SQ counters per pass).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/profbs
mkdir -p $OUT
C="GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- ./bin/otbench --bytes 4G --iters 3 --warmup 1 --inplace --mode ctr --impl bitslice > $OUT/kt.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/bs -o run -- ./bin/otbench --bytes 4G --iters 3 --warmup 1 --inplace --mode ctr --impl bitslice > $OUT/bs.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/tt -o run -- ./bin/otbench --bytes 4G --iters 3 --warmup 1 --inplace --mode ctr --impl ttable > $OUT/tt.log 2>&1
rc=$?
find $OUT -name '*.csv' | head; exit $rc
