#!/bin/bash
# Kernel-trace + stats of the final headline bench and of the batched CTR benchmark.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r1h
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/bench -o bench -- python3 bench.py --steps 5 --warmup 2 --no-clock > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/batch -o batch -- python3 benchmarks/batch_ctr.py --no-eager > $OUT/batch.log 2>&1 || { tail -20 $OUT/batch.log; exit 1; }
tail -1 $OUT/batch.log
find $OUT -name "*stats*.csv" | head
