#!/bin/bash
# The claimed split for CBC / CFB decryption of independent segments: GPU
# tests, then T-table vs split (4 KiB and 512 B segments), verified, with power.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r4_seg_split}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_faults.py -x -v --timeout 120 \
    --timeout-method thread -k "segment or split or decrypt or routing or fault" > $O/gpu_tests.log 2>&1 ||
    { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
B="--bytes 16G --iters 150 --warmup 3"
C=""
for m in cbc-dec-seg cfb-dec-seg; do for b in 256 128; do for sg in 4096 512; do
    C="$C;--mode $m --bits $b $B --seg $sg --impl ttable;--mode $m --bits $b $B --seg $sg --impl split"
done; done; done
bash scripts/ab_power.sh ${1:-r4_seg_split} 1 "${C#;}" base
