#!/bin/bash
# Kernel trace of the library's claimed split (ECB-256 / ECB-dec-256 64 GiB in
# place, CBC-dec-256 32 GiB): both kernels should start together and end
# together in every call (tools/split_timeline.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r4_claim_trace}
mkdir -p $O
for cfg in "ecb 64G --inplace" "ecb-dec 64G --inplace" "cbc-dec 32G" "ecb 4G --inplace"; do
    set -- $cfg
    n=$1_$2
    timeout -k 10 120 rocprofv3 --kernel-trace -d $O/db_$n -o run -- ./bin/otbench --mode $1 --bits 256 --bytes $2 $3 \
        --impl split --iters 6 --warmup 1 --verify > $O/run_$n.log 2>&1 || { tail -20 $O/run_$n.log; exit 1; }
    db=$(find $O/db_$n -name '*.db' | head -1)
    python3 tools/split_timeline.py "$db" --label "$n" | tee -a $O/timeline.txt || exit 1
done
