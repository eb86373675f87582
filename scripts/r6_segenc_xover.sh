#!/bin/bash
# Round 6: segment encryption, grid T-table kernel vs the persistent claim
# kernel (OTC_SEGENC_PERSISTENT_MIN_MIB=100000 / =1), 2 interleaved reps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r6/segenc_xover; mkdir -p $O
for rep in 1 2; do
  for arm in grid persistent; do
    [ $arm = grid ] && export OTC_SEGENC_PERSISTENT_MIN_MIB=100000 || export OTC_SEGENC_PERSISTENT_MIN_MIB=1
    for cfg in "cfb-enc-seg 128 2048" "cbc-enc-seg 128 4096" "cbc-enc-seg 256 4096" "cbc-enc-seg 256 512"; do
      for sz in 768M 1G 1280M 1536M 2G; do
        set -- $cfg
        timeout -k 10 60 ./bin/otbench --mode $1 --bits $2 --bytes $sz --seg $3 --iters 10 --warmup 2 \
            | sed "s|^{|{\"arm\": \"$arm\", \"rep\": $rep, \"seg\": $3, |" >> $O/ab.jsonl || { echo "FAILED $arm $cfg $sz"; exit 1; }
      done
    done
  done
done
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r6/segenc_xover/ab.jsonl") if l.startswith("{")]
by = collections.defaultdict(list)
for r in rows:
    by[(r["mode"], r["bits"], r["seg"], r["bytes"] >> 20, r["arm"])].append(r["gbps"])
for k in sorted(by):
    print(k, " ".join(f"{v:.1f}" for v in by[k]))
PY
