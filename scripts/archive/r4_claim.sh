#!/bin/bash
# The claimed split (both kernels take 2048-block units from one counter) vs
# the T-table alone and vs the static shares (otbench *-split, now joined per
# call): GPU tests first, then a verified A/B with power.
#   gpurun --timeout 1200 -- bash scripts/r4_claim.sh NAME
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r4_claim}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
    -k "split or decrypt or cfb or routing or concurrent" > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
I64="--bytes 64G --inplace --iters 60 --warmup 2"
I4="--bytes 4G --inplace --iters 500 --warmup 20"
O32="--bytes 32G --iters 100 --warmup 2"
C="--mode ecb --bits 256 $I64 --impl ttable;--mode ecb --bits 256 $I64 --impl split"
C="$C;--mode ecb-split --bits 256 $I64 --share 0.25;--mode ecb-split --bits 256 $I64 --share 0.35"
C="$C;--mode ecb --bits 256 $I4 --impl ttable;--mode ecb --bits 256 $I4 --impl split;--mode ecb-split --bits 256 $I4 --share 0.25"
C="$C;--mode ecb --bits 128 $I64 --impl ttable;--mode ecb --bits 128 $I64 --impl split;--mode ecb-split --bits 128 $I64 --share 0.2"
C="$C;--mode ecb-dec --bits 256 $I64 --impl ttable;--mode ecb-dec --bits 256 $I64 --impl split;--mode ecbdec-split --bits 256 $I64 --share 0.2"
C="$C;--mode ecb-dec --bits 128 $I64 --impl split"
C="$C;--mode cbc-dec --bits 256 $O32 --impl ttable;--mode cbc-dec --bits 256 $O32 --impl split;--mode cbcdec-split --bits 256 $O32 --share 0.15"
C="$C;--mode cfb-dec --bits 256 $O32 --impl ttable;--mode cfb-dec --bits 256 $O32 --impl split;--mode cfbdec-split --bits 256 $O32 --share 0.2"
bash scripts/ab_power.sh ${1:-r4_claim} 1 "$C" base
