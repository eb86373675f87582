#!/bin/bash
# One PMC pass (8 SQ + 1 GRBM counters) over the bitsliced bulk kernel of a
# 4 GiB in-place otbench run, summarised per kernel (run on the box):
#   bash scripts/pmc_bulk.sh NAME "--mode ctr --bits 128"
# -> gpurun_out/NAME/summary.txt: the bulk (full-task) launch, VALU per wave =
# per 2048-block task
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
name=$1
args=$2
O=gpurun_out/$name
mkdir -p $O
C="GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVES SQ_WAVE_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/db -o run -- \
    ./bin/otbench $args --bytes 4G --impl bitslice --inplace --iters 3 --warmup 1 > $O/run.log 2>&1 ||
    { tail -20 $O/run.log; exit 1; }
csv=$(find $O/db -name '*counter_collection.csv' | head -1)
python3 tools/pmc_summary.py --kernel "true>((anonymous namespace)::BsParams" "$csv" > $O/summary.txt && cat $O/summary.txt
