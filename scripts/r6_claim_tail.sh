#!/bin/bash
# Round 6: the persistent T-table claim kernel's start ramp and claim tail,
# from the wave-start / wave-end trace of a diagnostic build
# (make variant NAME=strace VFLAGS=-DOTC_SPLIT_TRACE=1), AES-128 ECB.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r6/claim_tail
mkdir -p $O
V=${V:-variants/strace}
for b in ${SIZES:-512M 1G 2G 8G}; do
  LD_LIBRARY_PATH=$V timeout -k 10 60 ./bin/otbench --mode ecb --bits 128 --bytes $b --impl ttable --iters 10 --warmup 3 \
      --strace >> $O/${TAG:-base}.log 2>&1 || { echo "FAILED $b"; tail $O/${TAG:-base}.log; exit 1; }
done
cat $O/${TAG:-base}.log
