#!/bin/bash
# Mode x key-size sweep of the current build (through gpurun):
#   gpurun --timeout 900 -- bash scripts/sweep.sh OUTNAME
# every AES mode at 128/192/256 bits on a 4 GiB buffer (impl auto; in place
# except the chained decrypts), every line verified against the oracle
# (otbench --verify: pre-op snapshots, so in place too; exit 3 on a mismatch),
# CTR at 64 GiB with both kernels, then the J/GB power probe and a kernel trace
# of a short bench.py run.  Output under gpurun_out/OUTNAME/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-sweep}; mkdir -p $O
for m in ctr ecb ecb-dec cbc-dec cfb-dec cbc-enc-seg cfb-enc-seg cbc-dec-seg cfb-dec-seg; do for b in 128 192 256; do
    ip=--inplace  # the chained decrypts read the previous ciphertext block: out of place
    case $m in cbc-dec|cfb-dec|cbc-dec-seg|cfb-dec-seg) ip= ;; esac
    timeout -k 10 120 ./bin/otbench --mode $m --bits $b --bytes 4G $ip --iters 100 --warmup 10 --clock --verify >> $O/sweep.jsonl || exit 1
done; done
# the ECB / decrypt paths at 64 GiB (32 GiB out of place for CBC), auto = the co-resident split
for m in ecb ecb-dec cbc-dec; do for b in 128 256; do
    sz=64G; ip=--inplace
    [ $m = cbc-dec ] && { sz=32G; ip=; }
    timeout -k 10 120 ./bin/otbench --mode $m --bits $b --bytes $sz $ip --iters 10 --warmup 2 --clock --verify >> $O/big.jsonl || exit 1
done; done
for i in ttable bitslice; do for b in 128 256; do
    timeout -k 10 120 ./bin/otbench --mode ctr --bits $b --bytes 64G --inplace --iters 10 --warmup 2 --impl $i --clock --verify >> $O/ctr64g.jsonl || exit 1
done; done
bash scripts/power_probe.sh "bitslice" > $O/power.txt 2>&1 || { tail -5 $O/power.txt; exit 1; }
cp -r gpurun_out/power $O/ 2>/dev/null
mkdir -p $O/kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt/db -o run -- python3 bench.py --steps 5 --warmup 1 --no-scatter --no-stream > $O/kt/run.log 2>&1 || { tail -20 $O/kt/run.log; exit 1; }
db=$(find $O/kt/db -name '*.db' | head -1)
python3 tools/rocpd_summary.py "$db" > $O/kt/kernels.txt && head -12 $O/kt/kernels.txt
python3 - "$O" <<'PY'
import json, sys
o = sys.argv[1]
for f in ("sweep.jsonl", "big.jsonl", "ctr64g.jsonl"):
    for l in open(f"{o}/{f}"):
        d = json.loads(l)
        print(f, d["mode"], d["bits"], d["bytes"] >> 30, "GiB", d["impl"], d["gbps"], d.get("held_clock_ghz"),
              "verified" if d["verified"] is True else "NOT VERIFIED")
PY
cat $O/power.txt | tail -3
