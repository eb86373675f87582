#!/bin/bash
# Rehearse bench.py's multi-rank path (2 ranks sharing the one GPU of the box:
# gloo for the host-side collectives, per-rank counter offsets, max over ranks).
set -o pipefail
export TMPDIR=/tmp OTC_DIST_BACKEND=gloo OTC_SHARE_GPUS=1
OUT=gpurun_out/dp2
mkdir -p $OUT
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --gib 8 > $OUT/bench_dp2.log 2>&1 || { tail -30 $OUT/bench_dp2.log; exit 1; }
grep '^{' $OUT/bench_dp2.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 benchmarks/cbc_scatter.py --gib-per-gpu 2 --chunk-mib 256 > $OUT/cbc_dp2.log 2>&1 || { tail -30 $OUT/cbc_dp2.log; exit 1; }
grep '^{' $OUT/cbc_dp2.log
