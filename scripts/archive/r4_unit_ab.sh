#!/bin/bash
# Claim unit A/B: the round-4 split with 2048-block units for both sides
# (variants/base = the default build) vs 1024-block T-table units with 2-unit
# bitsliced tasks (variants/unit1k: make variant NAME=unit1k
# VFLAGS=-DOTC_CLAIM_UNIT=1024u) and a reserve left to the T-table
# (OTC_SPLIT_RESERVE_MIB), against the T-table alone.  Verified, interleaved,
# 2 reps.  -> gpurun_out/OUT/ab.jsonl
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r4_unit_ab}
mkdir -p $O
run() { # label lib reserve args...
    local lab=$1 lib=$2 res=$3; shift 3
    local r
    r=$(OTC_SPLIT_RESERVE_MIB=$res LD_LIBRARY_PATH=variants/$lib timeout -k 10 150 ./bin/otbench "$@" --verify) || { echo "FAILED $lab $*"; exit 1; }
    echo "{\"label\": \"$lab\", \"r\": $r}" >> $O/ab.jsonl
    python3 - "$r" "$lab" <<'PY'
import json, sys
d = json.loads(sys.argv[1])
print(f'{sys.argv[2]:10s} {d["mode"]:8s} {d["bytes"] >> 20:6d} MiB {d["impl"]:7s} {d["gbps"]:8.1f} v={d["verified"]}', flush=True)
PY
}
for rep in 1 2; do
for sz in ${SIZES:-256M 1000M 4G}; do
    it=60; [ $sz = 256M ] && it=300; [ $sz = 1000M ] && it=150
    for m in ecb cbc-dec; do
        ip=--inplace; [ $m = cbc-dec ] && ip=
        A="--mode $m --bits 256 --bytes $sz $ip --iters $it --warmup 5"
        run ttable base 0 $A --impl ttable || exit 1
        run base base 0 $A --impl split || exit 1
        for R in ${RESERVES:-0 32 96 160}; do run unit1k_r$R unit1k $R $A --impl split || exit 1; done
    done
done
done
