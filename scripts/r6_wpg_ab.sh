#!/bin/bash
# Round 6: the bitsliced CTR launches with 1 / 2 / 4 waves per workgroup
# (variants/wpg1, wpg2; release = 4), 3 interleaved reps, 64 GiB in place
# (the bench shape) and 4 GiB; each variant verified first (odd size: edge
# tasks run).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r6/wpg; mkdir -p $O
B=our_tree_amd/lib
for lib in variants/wpg1 variants/wpg2; do
  for bits in 128 256; do
    LD_LIBRARY_PATH=$lib timeout -k 10 60 ./bin/otbench --mode ctr --bits $bits --bytes 2147487749 --iters 2 --warmup 1 \
        --verify >> $O/verify.jsonl 2>&1 || exit 1
  done
done
grep -q '"verified": false' $O/verify.jsonl && { echo "VERIFY FAILED"; exit 1; }
echo "verified: $(grep -c '"verified": true' $O/verify.jsonl)"
for rep in 1 2 3; do
  for lib in $B variants/wpg1 variants/wpg2; do
    for cfg in "128 64G" "256 64G" "128 4G"; do
      set -- $cfg
      LD_LIBRARY_PATH=$lib timeout -k 10 90 ./bin/otbench --mode ctr --bits $1 --bytes $2 --inplace --iters 10 --warmup 2 --clock \
          | sed "s|^{|{\"lib\": \"$lib\", \"rep\": $rep, |" >> $O/ab.jsonl || exit 1
    done
  done
done
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r6/wpg/ab.jsonl") if l.startswith("{")]
by = collections.defaultdict(list)
for r in rows:
    by[(r["bits"], r["bytes"] >> 30, r["lib"])].append(f'{r["gbps"]:.1f}@{r.get("held_clock_ghz") or 0:.2f}')
for k in sorted(by):
    print(k, " ".join(by[k]))
PY
