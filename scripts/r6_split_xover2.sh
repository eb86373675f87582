#!/bin/bash
# Round 6, after the first-claim fix: the co-resident split (impl split) vs
# the persistent T-table claim kernel alone (auto below 2 GiB) at 1-2 GiB,
# 2 interleaved reps, one box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r6/split_xover2; mkdir -p $O
for rep in 1 2; do
  for impl in auto split; do
    for cfg in "ecb 128" "ecb 256" "cbc-dec 128" "ecb-dec 256" "cfb-dec 256"; do
      for sz in 768M 1G 1536M; do
        set -- $cfg
        timeout -k 10 60 ./bin/otbench --mode $1 --bits $2 --bytes $sz --impl $impl --iters 15 --warmup 3 \
            | sed "s|^{|{\"rep\": $rep, |" >> $O/ab.jsonl || { echo "FAILED $impl $cfg $sz"; exit 1; }
      done
    done
  done
done
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r6/split_xover2/ab.jsonl") if l.startswith("{")]
by = collections.defaultdict(list)
for r in rows:
    by[(r["mode"], r["bits"], r["bytes"] >> 20, r["ran"])].append(r["gbps"])
for k in sorted(by):
    print(k, " ".join(f"{v:.1f}" for v in by[k]))
PY
