#!/bin/bash
# Round 6: after the persistent T-table CTR kernel, CTR at the bench shape
# (64 GiB in place): bitsliced vs persistent T-table vs the old static grid
# (OTC_TT_CTR_PERSISTENT_MIN_MIB=1000000), with socket energy over each
# timed loop (tools/power_run.py), 2 interleaved reps, AES-128 and AES-256.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r6/ctr64; mkdir -p $O
for rep in 1 2; do
  for arm in bitslice persist grid; do
    for bits in 128 256; do
      impl=ttable; [ $arm = bitslice ] && impl=bitslice
      if [ $arm = grid ]; then export OTC_TT_CTR_PERSISTENT_MIN_MIB=1000000; else unset OTC_TT_CTR_PERSISTENT_MIN_MIB; fi
      timeout -k 10 120 python3 tools/power_run.py --label "$arm" -- ./bin/otbench --mode ctr --bits $bits --bytes 64G --impl $impl \
          --inplace --iters 60 --warmup 3 --mark | sed "s|^{|{\"arm\": \"$arm\", \"rep\": $rep, |" >> $O/ab.jsonl || exit 1
    done
  done
done
unset OTC_TT_CTR_PERSISTENT_MIN_MIB
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r6/ctr64/ab.jsonl") if l.startswith("{")]
by = collections.defaultdict(list)
for r in rows:
    p = r.get("power") or {}
    by[(r["bits"], r["arm"])].append(f'{r["gbps"]:.1f} GB/s {r.get("joules_per_gb") or 0:.3f} J/GB {p.get("avg_socket_w") or 0:.0f} W')
for k in sorted(by):
    print(k, " | ".join(by[k]))
PY
