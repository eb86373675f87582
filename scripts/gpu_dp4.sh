#!/bin/bash
# GPU tests on the current build, then bench.py's multi-rank path rehearsed at
# 4 ranks sharing the box's one GPU (gloo host collectives, per-rank counter
# offsets, max over ranks; throughput meaningless), then the default bench.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/dp4
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
OTC_DIST_BACKEND=gloo OTC_SHARE_GPUS=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 3 --warmup 1 --gib 4 > $OUT/bench_dp4.txt 2>&1 || { tail -30 $OUT/bench_dp4.txt; exit 1; }
grep '^{' $OUT/bench_dp4.txt
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err.txt || { tail -20 $OUT/bench.err.txt; exit 1; }
cat $OUT/bench.json
