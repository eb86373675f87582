#!/bin/bash
# CTR split with half the bitsliced workgroups (one per two CUs, variant half;
# half also routes CTR >= 8 GiB to the split for the bench run) vs base.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=${1:-r5_ctr_half}; mkdir -p gpurun_out/$O
C="--mode ctr --bits 128 --bytes 64G --inplace --iters 10 --impl split --split-stats;--mode ctr --bits 256 --bytes 64G --inplace --iters 10 --impl split --split-stats;--mode ctr --bits 128 --bytes 64G --inplace --iters 10 --impl bitslice"
bash scripts/ab_power.sh $O 1 "$C" base half || exit 1
OTC_LIB=variants/half/libotc.so timeout -k 10 300 python3 tools/split_queue_check.py --streams 12 --gib 16 > gpurun_out/$O/check12_half.jsonl 2>&1; cat gpurun_out/$O/check12_half.jsonl
OTC_LIB=variants/half/libotc.so timeout -k 10 600 python3 bench.py --no-stream --no-scatter --no-refmethod > gpurun_out/$O/bench_half.json 2> gpurun_out/$O/bench_half.err; tail -c 200 gpurun_out/$O/bench_half.json
