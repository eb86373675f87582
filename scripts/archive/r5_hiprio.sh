#!/bin/bash
# Split stream placement: both halves CU-masked (base) vs T-table on the
# caller's stream + bitsliced half on a non-blocking highest-priority stream
# (hiprio): otbench (null stream), a 12-stream torch process, and bench.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=${1:-r5_hiprio}; mkdir -p gpurun_out/$O
C="--mode ecb --bits 256 --bytes 64G --inplace --iters 10 --split-stats;--mode cbc-dec --bits 256 --bytes 16G --iters 10 --split-stats;--mode ctr --bits 128 --bytes 64G --inplace --iters 10 --impl split --split-stats;--mode ctr --bits 256 --bytes 64G --inplace --iters 10 --impl split --split-stats;--mode ctr --bits 128 --bytes 64G --inplace --iters 10 --impl bitslice"
bash scripts/ab_power.sh $O 1 "$C" base hiprio || exit 1
for v in base hiprio; do
    LD_LIBRARY_PATH=variants/$v OTC_LIB=variants/$v/libotc.so timeout -k 10 300 python3 tools/split_queue_check.py --streams 12 --gib 16 > gpurun_out/$O/check12_$v.jsonl 2>&1
    echo "== $v"; cat gpurun_out/$O/check12_$v.jsonl
done
