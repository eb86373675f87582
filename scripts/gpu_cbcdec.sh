#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/cbcdec
mkdir -p $OUT
timeout -k 10 300 python -u benchmarks/cbc_scatter.py --gib-per-gpu 8 --decrypt > $OUT/dec_1gpu.log 2>&1 || { tail -20 $OUT/dec_1gpu.log; exit 1; }
grep '^{' $OUT/dec_1gpu.log
OTC_DIST_BACKEND=gloo OTC_SHARE_GPUS=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29541 benchmarks/cbc_scatter.py --gib-per-gpu 1 --chunk-mib 128 --decrypt > $OUT/dec_dp3.log 2>&1 || { tail -30 $OUT/dec_dp3.log; exit 1; }
grep '^{' $OUT/dec_dp3.log
