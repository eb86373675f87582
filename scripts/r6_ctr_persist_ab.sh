#!/bin/bash
# Round 6: CTR on the T-table from 512 MiB as a persistent claim kernel vs the
# grid kernel (OTC_TT_CTR_PERSISTENT_MIN_MIB=100000), and the bitsliced kernel
# beside both at 1-2 GiB (the auto threshold), 3 interleaved reps; the new
# path verified and its GPU test first.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r6/ctr_persist; mkdir -p $O
for cfg in "128 700M" "256 513M" "192 1500M"; do
  set -- $cfg
  timeout -k 10 60 ./bin/otbench --mode ctr --bits $1 --bytes $2 --impl ttable --iters 2 --warmup 1 --verify >> $O/verify.jsonl 2>&1 || exit 1
done
grep -q '"verified": false' $O/verify.jsonl && { echo "VERIFY FAILED"; exit 1; }
echo "verified: $(grep -c '"verified": true' $O/verify.jsonl)"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "ctr" \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
  for arm in grid persist bitslice; do
    for cfg in "128 512M" "128 768M" "128 1G" "128 1536M" "128 2G" "256 768M"; do
      set -- $cfg
      impl=ttable; [ $arm = bitslice ] && impl=bitslice
      if [ $arm = grid ]; then export OTC_TT_CTR_PERSISTENT_MIN_MIB=100000; else unset OTC_TT_CTR_PERSISTENT_MIN_MIB; fi
      timeout -k 10 60 ./bin/otbench --mode ctr --bits $1 --bytes $2 --impl $impl --iters 20 --warmup 3 \
          | sed "s|^{|{\"arm\": \"$arm\", \"rep\": $rep, |" >> $O/ab.jsonl || exit 1
    done
  done
done
unset OTC_TT_CTR_PERSISTENT_MIN_MIB
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r6/ctr_persist/ab.jsonl") if l.startswith("{")]
by = collections.defaultdict(list)
for r in rows:
    by[(r["bits"], r["bytes"] >> 20, r["arm"])].append(r["gbps"])
for k in sorted(by):
    print(k, " ".join(f"{v:.1f}" for v in by[k]))
PY
