#!/bin/bash
# Second share sweep: CFB-dec and CBC-dec splits at the low shares, verified,
# with power (the current build as variants/base).
#   gpurun --timeout 900 -- bash scripts/r4_shares.sh NAME
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
B32="--bytes 32G --iters 100 --warmup 2"
B4="--bytes 4G --iters 700 --warmup 20"
C=""
for b in 256 128; do
    for s in 0.1 0.15 0.2; do C="$C;--mode cfbdec-split --bits $b $B32 --share $s;--mode cfbdec-split --bits $b $B4 --share $s"; done
    for s in 0.1 0.15 0.2; do C="$C;--mode cbcdec-split --bits $b $B32 --share $s"; done
    C="$C;--mode cbc-dec --bits $b $B32 --impl ttable;--mode cfb-dec --bits $b $B32 --impl ttable"
done
bash scripts/ab_power.sh ${1:-r4_shares} 1 "${C#;}" base
