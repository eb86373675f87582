#!/bin/bash
# Co-residency of the claimed splits after the descriptor fix (dynamic LDS in
# the T-table claim kernels, csrc/hip/aes_tt.hip tt_lds):
#  1. wave-start trace (variants/strace, OTC_SPLIT_TRACE) + the units each
#     side took, every split mode at AES-256 4 GiB;
#  2. split vs T-table vs bitsliced alone, with power (scripts/ab_power.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r5_cores}
mkdir -p $O
for m in ${MODES:-ecb ecb-dec cbc-dec cfb-dec "cbc-enc-seg --seg 4096" "cbc-enc-seg --seg 512" "cfb-enc-seg --seg 4096"}; do
    echo "== $m" | tee -a $O/trace.txt
    LD_LIBRARY_PATH=variants/strace timeout -k 10 60 ./bin/otbench --mode $m --bits 256 --bytes 4G --impl split \
        --iters 3 --warmup 1 --split-stats --strace >> $O/trace.txt 2>&1 || { tail -20 $O/trace.txt; exit 1; }
    tail -3 $O/trace.txt
done
B="--bits 256 --bytes 4G --iters ${ITERS:-30} --split-stats"
C=""
for m in ${MODES:-ecb ecb-dec cbc-dec cfb-dec "cbc-enc-seg --seg 4096" "cbc-enc-seg --seg 512" "cfb-enc-seg --seg 4096"}; do
    for i in split ttable bitslice; do C="$C;--mode $m --impl $i $B"; done
done
bash scripts/ab_power.sh ${1:-r5_cores} 1 "${C#;}" base
