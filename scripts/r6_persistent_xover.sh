#!/bin/bash
# Round 6: with the first claim units handed out, where does the persistent
# T-table claim kernel start to beat the grid T-table kernel?  Arms: the
# default thresholds (grid below 896 MiB; segment encryption below 1-2 GiB)
# vs the persistent kernel at every size (OTC_TT_PERSISTENT_MIN_MIB=1,
# OTC_SEGENC_PERSISTENT_MIN_MIB=1), 2 interleaved reps, one box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r6/xover; mkdir -p $O
for m in ecb cbc-dec; do
  OTC_TT_PERSISTENT_MIN_MIB=1 timeout -k 10 60 ./bin/otbench --mode $m --bits 128 --bytes 129M --iters 2 --warmup 1 --verify \
      >> $O/verify.jsonl 2>&1 || { echo "VERIFY FAILED $m"; exit 1; }
done
OTC_SEGENC_PERSISTENT_MIN_MIB=1 timeout -k 10 60 ./bin/otbench --mode cbc-enc-seg --bits 256 --bytes 257M --seg 4096 --iters 2 \
    --warmup 1 --verify >> $O/verify.jsonl 2>&1 || { echo "VERIFY FAILED seg"; exit 1; }
grep -q '"verified": false' $O/verify.jsonl && { echo "A VERIFICATION FAILED"; exit 1; }
for rep in 1 2; do
  for arm in default persistent; do
    for cfg in "ecb 128" "ecb 256" "cbc-dec 128" "ecb-dec 256"; do
      for sz in 128M 256M 512M 768M; do
        set -- $cfg
        if [ $arm = persistent ]; then export OTC_TT_PERSISTENT_MIN_MIB=1; else unset OTC_TT_PERSISTENT_MIN_MIB; fi
        timeout -k 10 60 ./bin/otbench --mode $1 --bits $2 --bytes $sz --iters 30 --warmup 5 \
            | sed "s|^{|{\"arm\": \"$arm\", \"rep\": $rep, |" >> $O/ab.jsonl || { echo "FAILED $arm $cfg $sz"; exit 1; }
      done
    done
    unset OTC_TT_PERSISTENT_MIN_MIB
    for sz in 512M 1G 1536M; do
      if [ $arm = persistent ]; then export OTC_SEGENC_PERSISTENT_MIN_MIB=1; else unset OTC_SEGENC_PERSISTENT_MIN_MIB; fi
      timeout -k 10 60 ./bin/otbench --mode cbc-enc-seg --bits 256 --bytes $sz --seg 4096 --iters 20 --warmup 3 \
          | sed "s|^{|{\"arm\": \"$arm\", \"rep\": $rep, |" >> $O/ab.jsonl || { echo "FAILED seg $arm $sz"; exit 1; }
    done
    unset OTC_SEGENC_PERSISTENT_MIN_MIB
  done
done
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r6/xover/ab.jsonl") if l.startswith("{")]
by = collections.defaultdict(list)
for r in rows:
    by[(r["mode"], r["bits"], r["bytes"] >> 20, r["arm"])].append(r["gbps"])
for k in sorted(by):
    print(k, " ".join(f"{v:.1f}" for v in by[k]))
PY
