#!/bin/bash
# Bitsliced CFB128 decryption and its co-resident split: GPU tests, then a
# verified share sweep with power (scripts/ab_power.sh, the current build as
# variants/base), plus CBC-dec after the IV-blend change (no private IV copy).
#   gpurun --timeout 1200 -- bash scripts/r4_cfb.sh NAME
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r4_cfb}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
    -k "cfb or decrypt or split or routing or beyond" > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
B32="--bytes 32G --iters 100 --warmup 2"
B4="--bytes 4G --iters 700 --warmup 20"
C=""
for b in 256 128; do
    C="$C;--mode cfb-dec --bits $b $B32 --impl ttable;--mode cfb-dec --bits $b $B32 --impl bitslice"
    for s in 0.2 0.25 0.3 0.35; do C="$C;--mode cfbdec-split --bits $b $B32 --share $s"; done
    C="$C;--mode cfb-dec --bits $b $B4 --impl ttable"
    for s in 0.2 0.25 0.3; do C="$C;--mode cfbdec-split --bits $b $B4 --share $s"; done
done
C="$C;--mode cbc-dec --bits 256 $B32 --impl bitslice;--mode cbc-dec --bits 256 $B32 --impl split"
bash scripts/ab_power.sh ${1:-r4_cfb} 1 "${C#;}" base
