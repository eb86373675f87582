#!/bin/bash
# bench.py's multi-rank path rehearsed at 8 ranks (the driver's largest N)
# sharing the box's one GPU: gloo host collectives, per-rank counter offsets
# and verification, max over ranks, one JSON line from rank 0.  Throughput is
# meaningless here (8 ranks time-share one GPU); the 8-GPU numbers come from
# the driver's own node runs.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/dp8
mkdir -p $OUT
OTC_DIST_BACKEND=gloo OTC_SHARE_GPUS=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29543 bench.py --gpus 8 --steps 3 --warmup 1 --gib 2 --no-clock > $OUT/bench_dp8.txt 2>&1 || { tail -30 $OUT/bench_dp8.txt; exit 1; }
grep '^{' $OUT/bench_dp8.txt
