#!/bin/bash
# RCCL (nccl backend) code paths on the one-GPU box: world-size-1 RCCL groups.
set -o pipefail
mkdir -p gpurun_out/rccl1
export MASTER_ADDR=127.0.0.1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dist.py \
  > gpurun_out/rccl1/pytest.log 2>&1 &&
OTC_DIST_FORCE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --steps 3 --warmup 1 --gib 8 \
  > gpurun_out/rccl1/bench_torchrun_rccl.json 2> gpurun_out/rccl1/bench.err &&
OTC_DIST_FORCE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29532 benchmarks/cbc_scatter.py --gib-per-gpu 4 \
  > gpurun_out/rccl1/cbc_scatter_rccl.json 2> gpurun_out/rccl1/cbc.err &&
OTC_DIST_FORCE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29533 benchmarks/cbc_scatter.py --gib-per-gpu 4 --decrypt \
  > gpurun_out/rccl1/cbc_scatter_dec_rccl.json 2>> gpurun_out/rccl1/cbc.err
rc=$?
tail -3 gpurun_out/rccl1/pytest.log; cat gpurun_out/rccl1/*.json
exit $rc
