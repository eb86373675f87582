#!/bin/bash
# Where does the claimed split start to pay?  ECB-256 / ECB-dec-256 / CBC-dec-256
# T-table vs split from 16 MiB to 1 GiB, verified.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r4_small_split}
mkdir -p $O
for sz in ${SIZES:-64M 256M 512M 1000M 2G}; do
    for m in ecb ecb-dec cbc-dec; do
        ip=--inplace; [ $m = cbc-dec ] && ip=
        for i in ttable split; do
            timeout -k 10 120 ./bin/otbench --mode $m --bits 256 --bytes $sz $ip --impl $i --iters 200 --warmup 10 --verify \
                >> $O/small.jsonl || exit 1
        done
    done
done
for sz in 64M; do for i in ttable bitslice; do
    timeout -k 10 120 ./bin/otbench --mode ctr --bits 128 --bytes $sz --inplace --impl $i --iters 200 --warmup 10 --verify \
        >> $O/small.jsonl || exit 1
done; done
python3 - $O/small.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(f'{d["mode"]:8s} {d["bytes"] >> 20:6d} MiB {d["impl"]:7s} {d["gbps"]:8.1f} GB/s {d["verified"]}')
PY
