#!/bin/bash
# Wave-start trace of the final split (diagnostic build OTC_SPLIT_TRACE):
# when each kernel's waves started, and the units each side took.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r5_strace_final}; mkdir -p $O
for m in "ecb --bytes 4G --inplace" "ecb-dec --bytes 4G" "cbc-dec --bytes 4G" "cfb-dec --bytes 4G" "ctr --bytes 4G --inplace --impl split"; do
    echo "== $m" | tee -a $O/trace.txt
    LD_LIBRARY_PATH=variants/strace timeout -k 10 60 ./bin/otbench --mode $m --bits 256 --iters 3 --warmup 1 --split-stats --strace >> $O/trace.txt 2>&1 || { tail -20 $O/trace.txt; exit 1; }
done
cat $O/trace.txt
