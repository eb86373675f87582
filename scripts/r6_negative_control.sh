#!/bin/bash
# Round 6 final tree: the co-residency GPU test must PASS on the release and
# FAIL on the padded-descriptor build (variants/padclaim, round 4's defect),
# now that every wave's first unit is handed out (the serialised bitsliced
# half still gets only its pre-assigned 1.6% of a 2 GiB call, below the 5% bar).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
D=gpurun_out/r6/negctl; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_queues.py \
    -k coresident > $D/release.log 2>&1 || { echo "RELEASE FAILED"; tail -20 $D/release.log; exit 1; }
tail -1 $D/release.log
OTC_LIB=variants/padclaim/libotc.so timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread \
    tests/test_gpu_queues.py -k coresident > $D/padclaim.log 2>&1 && { echo "PADCLAIM UNEXPECTEDLY PASSED"; exit 1; }
tail -1 $D/padclaim.log
grep -m3 "AssertionError\|assert " $D/padclaim.log || true
