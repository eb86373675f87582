#!/bin/bash
# Kernel trace of the claimed splits (do both kernels co-run?):
# ECB-256 4 GiB in place, CBC-enc-seg-256 4 GiB (4 KiB segments).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r5_split_trace}
mkdir -p $O
for cfg in "ecb 4G" "cbc-enc-seg 4G"; do
    set -- $cfg
    n=$1_$2
    timeout -k 10 120 rocprofv3 --kernel-trace -d $O/db_$n -o run -- ./bin/otbench --mode $1 --bits 256 --bytes $2 --inplace \
        --impl split --iters 6 --warmup 1 --split-stats > $O/run_$n.log 2>&1 || { tail -20 $O/run_$n.log; exit 1; }
    db=$(find $O/db_$n -name '*.db' | head -1)
    python3 tools/split_timeline.py "$db" --label "$n" | tee -a $O/timeline.txt || exit 1
    python3 tools/rocpd_summary.py "$db" > $O/kernels_$n.txt
done
