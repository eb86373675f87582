#!/bin/bash
# Kernel trace of the co-resident split at several shares: per call, when the
# T-table and the bitsliced kernels start and end (tools/split_timeline.py).
#   gpurun --timeout 900 -- bash scripts/r4_split_trace.sh NAME
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r4_split_trace}
mkdir -p $O
for cfg in "ecb-split 256 64G --inplace" "ecb-split 256 4G --inplace" "ecbdec-split 256 64G --inplace"; do
    set -- $cfg
    for s in 0.1 0.15 0.2 0.25 0.3 0.35; do
        n=$1_$2_$3_$s
        timeout -k 10 120 rocprofv3 --kernel-trace -d $O/db_$n -o run -- ./bin/otbench --mode $1 --bits $2 --bytes $3 $4 \
            --share $s --iters 6 --warmup 1 > $O/run_$n.log 2>&1 || { tail -20 $O/run_$n.log; exit 1; }
        db=$(find $O/db_$n -name '*.db' | head -1)
        python3 tools/split_timeline.py "$db" --label "$n" | tee -a $O/timeline.txt || exit 1
    done
done
