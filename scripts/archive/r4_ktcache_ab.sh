#!/bin/bash
# Key-table cache A/B: the split with the bitsliced key-term table cached per
# key vs the per-call table (OTC_BS_KT_CACHE=0) vs the previous library
# (variants/base), and the T-table alone.  AES-256, verified, interleaved, 2
# reps; then a kernel trace of 256 MiB calls.  The cache was not adopted: build
# our_tree_amd/lib with profiles/r4/ktcache/ktcache.patch applied to rerun.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r4_ktcache_ab}
mkdir -p $O
run() { # label lib cache args...
    local lab=$1 lib=$2 c=$3; shift 3
    local r
    r=$(OTC_BS_KT_CACHE=$c LD_LIBRARY_PATH=$lib timeout -k 10 150 ./bin/otbench "$@" --verify) || { echo "FAILED $lab $*"; exit 1; }
    echo "{\"label\": \"$lab\", \"r\": $r}" >> $O/ab.jsonl
    python3 - "$r" "$lab" <<'PY'
import json, sys
d = json.loads(sys.argv[1])
print(f'{sys.argv[2]:10s} {d["mode"]:8s} {d["bytes"] >> 20:6d} MiB {d["impl"]:7s} {d["gbps"]:8.1f} v={d["verified"]}', flush=True)
PY
}
for rep in 1 2; do
for sz in ${SIZES:-256M 512M 1000M 4G}; do
    it=60; [ $sz = 256M ] && it=300; [ $sz = 512M ] && it=200; [ $sz = 1000M ] && it=150
    for m in ecb cbc-dec; do
        ip=--inplace; [ $m = cbc-dec ] && ip=
        A="--mode $m --bits 256 --bytes $sz $ip --iters $it --warmup 5"
        run ttable our_tree_amd/lib 1 $A --impl ttable || exit 1
        run base variants/base 1 $A --impl split || exit 1
        run percall our_tree_amd/lib 0 $A --impl split || exit 1
        run cached our_tree_amd/lib 1 $A --impl split || exit 1
    done
done
done
SIZE=256M timeout -k 10 200 bash scripts/r4_split_gaps.sh ${1:-r4_ktcache_ab}/trace_256m > /dev/null && tail -1 $O/trace_256m/timeline.txt
