#!/bin/bash
# Round 6: claim kernels with pre-assigned first units (the release) vs
# every unit claimed (${ARM:-variants/nopre}), interleaved reps, one box.  First:
# every claimed form verified on the release -- T-table alone (1 GiB + an odd
# remainder), split (2 GiB + odd), bitsliced alone (impl bitslice), segment
# encryption / decryption -- and the split / queue GPU tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r6/${OUT:-preassign}
mkdir -p $O
B=our_tree_amd/lib
V() { LD_LIBRARY_PATH=$B timeout -k 10 60 ./bin/otbench "$@" --iters 2 --warmup 1 --verify >> $O/verify.jsonl 2>&1 ||
      { echo "VERIFY FAILED $*"; tail -5 $O/verify.jsonl; exit 1; }; }
for m in ecb ecb-dec cbc-dec cfb-dec; do
  V --mode $m --bits 128 --bytes 1048578048
  V --mode $m --bits 256 --bytes 2147485696
  V --mode $m --bits 128 --bytes 1048578048 --impl bitslice
done
V --mode cbc-enc-seg --bits 256 --bytes 2G --seg 4096
V --mode cfb-enc-seg --bits 128 --bytes 1G --seg 512
V --mode cbc-dec-seg --bits 256 --bytes 2G --seg 4096
V --mode cfb-dec-seg --bits 128 --bytes 2G --seg 4096
echo "verified: $(grep -c '"verified": true' $O/verify.jsonl) of $(grep -c '^{' $O/verify.jsonl)"
grep -q '"verified": false' $O/verify.jsonl && { echo "A VERIFICATION FAILED"; exit 1; }
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_queues.py \
    tests/test_gpu_kernels.py -k "split or claim or coresid or persistent or seg or ecb or dec" > $O/pytest.log 2>&1 ||
    { echo "PYTEST FAILED"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
  for lib in ${ARM:-variants/nopre} $B; do
    for cfg in "ecb 128 1G" "ecb 256 1G" "cbc-dec 128 1G" "ecb 128 2G" "ecb 256 8G" "cbc-enc-seg 256 2G"; do
      set -- $cfg
      extra=""; [ $1 = cbc-enc-seg ] && extra="--seg 4096"
      LD_LIBRARY_PATH=$lib timeout -k 10 60 ./bin/otbench --mode $1 --bits $2 --bytes $3 $extra --iters 20 --warmup 3 \
          | sed "s|^{|{\"lib\": \"$lib\", \"rep\": $rep, |" >> $O/ab.jsonl || { echo "FAILED $lib $cfg"; exit 1; }
    done
  done
done
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r6/" + __import__("os").environ.get("OUT", "preassign") + "/ab.jsonl") if l.startswith("{")]
by = collections.defaultdict(list)
for r in rows:
    by[(r["mode"], r["bits"], r["bytes"] >> 20, r["ran"], r["lib"])].append(r["gbps"])
for k in sorted(by):
    print(k, " ".join(f"{v:.1f}" for v in by[k]))
PY
[ -d variants/strace ] && LD_LIBRARY_PATH=variants/strace timeout -k 10 60 ./bin/otbench --mode ecb --bits 128 --bytes 1G --impl ttable --iters 10 \
    --warmup 3 --strace > $O/trace.log 2>&1 && grep strace $O/trace.log || true
