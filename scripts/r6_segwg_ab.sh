#!/bin/bash
# Round 6: segment encryption below the persistent kernel's 1 GiB -- the grid
# kernel with workgroups sized to spread the chains over every CU (release)
# vs 1024-thread workgroups on nseg / 1024 CUs (variants/segfixed), 3
# interleaved reps; the release verified first, GPU segment tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r6/segwg; mkdir -p $O
B=our_tree_amd/lib
for cfg in "cbc-enc-seg 256 100M 4096" "cfb-enc-seg 128 300M 2048" "cbc-enc-seg 128 700M 512" "cbc-enc-seg 256 5M 4096"; do
  set -- $cfg
  LD_LIBRARY_PATH=$B timeout -k 10 60 ./bin/otbench --mode $1 --bits $2 --bytes $3 --seg $4 --iters 2 --warmup 1 --verify \
      >> $O/verify.jsonl 2>&1 || exit 1
done
grep -q '"verified": false' $O/verify.jsonl && { echo "VERIFY FAILED"; exit 1; }
echo "verified: $(grep -c '"verified": true' $O/verify.jsonl)"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "seg" \
    > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
  for lib in variants/segfixed $B; do
    for cfg in "256 64M 4096" "256 256M 4096" "256 768M 4096" "128 512M 4096" "256 512M 512" "128 256M 2048"; do
      set -- $cfg
      LD_LIBRARY_PATH=$lib timeout -k 10 60 ./bin/otbench --mode cbc-enc-seg --bits $1 --bytes $2 --seg $3 --iters 20 --warmup 3 \
          | sed "s|^{|{\"lib\": \"$lib\", \"rep\": $rep, \"seg\": $3, |" >> $O/ab.jsonl || exit 1
    done
  done
done
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r6/segwg/ab.jsonl") if l.startswith("{")]
by = collections.defaultdict(list)
for r in rows:
    by[(r["bits"], r["seg"], r["bytes"] >> 20, r["lib"])].append(r["gbps"])
for k in sorted(by):
    print(k, " ".join(f"{v:.1f}" for v in by[k]))
PY
