#!/bin/bash
# ARCHIVED: ran against the guided-claim build (256-block units, up to 8 per
# claim) and a variant holding the old rule; the guided code was reverted
# (docs/PERF.md round 6, profiles/r6/claim_tail/).
# Round 6: the persistent T-table claim kernel alone (auto for ECB / the
# decryptions at [896 MiB, 2 GiB)) with guided 256-block claims (the
# release) vs one 2048-block unit per claim (variants/unit2048, the old
# rule), interleaved reps, one box; every mode verified on the release first
# (an odd block count leaves a remainder past the last unit); then the
# wave-end trace of both rules (variants/strace has the new one).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r6/claim_guided
mkdir -p $O
B=our_tree_amd/lib
for m in ecb ecb-dec cbc-dec cfb-dec; do
  for bits in 128 256; do
    LD_LIBRARY_PATH=$B timeout -k 10 60 ./bin/otbench --mode $m --bits $bits --bytes 1048578048 --iters 2 --warmup 1 --verify \
        >> $O/verify.jsonl 2>&1 || { echo "VERIFY FAILED $m $bits"; tail -5 $O/verify.jsonl; exit 1; }
  done
done
grep -c '"verified": true' $O/verify.jsonl
for rep in 1 2 3; do
  for lib in variants/unit2048 $B; do
    for cfg in "ecb 128 1G" "ecb 256 1G" "ecb 128 1536M" "ecb-dec 128 1G" "cbc-dec 128 1G" "cfb-dec 256 1G"; do
      set -- $cfg
      LD_LIBRARY_PATH=$lib timeout -k 10 60 ./bin/otbench --mode $1 --bits $2 --bytes $3 --iters 20 --warmup 3 \
          | sed "s|^{|{\"lib\": \"$lib\", \"rep\": $rep, |" >> $O/ab.jsonl || { echo "FAILED $lib $cfg"; exit 1; }
    done
  done
done
for v in variants/strace; do
  LD_LIBRARY_PATH=$v timeout -k 10 60 ./bin/otbench --mode ecb --bits 128 --bytes 1G --impl ttable --iters 10 --warmup 3 \
      --strace > $O/trace_guided.log 2>&1 || exit 1
done
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r6/claim_guided/ab.jsonl") if l.startswith("{")]
by = collections.defaultdict(list)
for r in rows:
    by[(r["mode"], r["bits"], r["bytes"] >> 20, r["lib"])].append(r["gbps"])
for k in sorted(by):
    print(k, " ".join(f"{v:.1f}" for v in by[k]))
PY
cat $O/trace_guided.log | grep strace
