#!/bin/bash
# ARCHIVED: the A/B arm (variants/twomemset, OTC_CLAIM_TWO_MEMSETS) was removed
# after this run (profiles/r6/claim_tail/one_fill_ab.jsonl).
# Round 6: one claim-counter fill per call (the release) vs two
# (variants/twomemset), 3 interleaved reps, mid sizes where a few us count;
# the release verified on every claimed form first.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r6/memset; mkdir -p $O
B=our_tree_amd/lib
for cfg in "ecb 128 600M" "ecb-dec 256 2049M" "cbc-dec 128 1G --impl bitslice" "cfb-dec 256 2G"; do
  set -- $cfg; LD_LIBRARY_PATH=$B timeout -k 10 60 ./bin/otbench --mode $1 --bits $2 --bytes $3 ${4:+$4 $5} --iters 2 --warmup 1 --verify >> $O/verify.jsonl 2>&1 || exit 1
done
grep -q '"verified": false' $O/verify.jsonl && { echo "VERIFY FAILED"; exit 1; }
echo "verified: $(grep -c '"verified": true' $O/verify.jsonl)"
for rep in 1 2 3; do
  for lib in variants/twomemset $B; do
    for cfg in "ecb 128 512M" "ecb 256 512M" "cbc-dec 128 768M" "ecb 128 1G" "ecb 128 2G"; do
      set -- $cfg
      LD_LIBRARY_PATH=$lib timeout -k 10 60 ./bin/otbench --mode $1 --bits $2 --bytes $3 --iters 30 --warmup 5 \
          | sed "s|^{|{\"lib\": \"$lib\", \"rep\": $rep, |" >> $O/ab.jsonl || exit 1
    done
  done
done
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r6/memset/ab.jsonl") if l.startswith("{")]
by = collections.defaultdict(list)
for r in rows:
    by[(r["mode"], r["bits"], r["bytes"] >> 20, r["ran"], r["lib"])].append(r["gbps"])
for k in sorted(by):
    print(k, " ".join(f"{v:.1f}" for v in by[k]))
PY
