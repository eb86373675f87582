set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6/xover_new; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for cfg in "ecb 128 512M" "ecb 128 768M" "ecb 256 600M" "cbc-dec 128 768M" "ecb-dec 256 512M" "cfb-dec 128 700M"; do
  set -- $cfg
  timeout -k 10 60 ./bin/otbench --mode $1 --bits $2 --bytes $3 --iters 10 --warmup 2 --verify >> $O/auto.jsonl 2>&1 || exit 1
done
for sz in 1G 1536M; do
  timeout -k 10 60 ./bin/otbench --mode cbc-enc-seg --bits 256 --bytes $sz --seg 4096 --iters 10 --warmup 2 --verify >> $O/auto.jsonl 2>&1 || exit 1
  timeout -k 10 60 ./bin/otbench --mode cfb-enc-seg --bits 128 --bytes $sz --seg 2048 --iters 10 --warmup 2 --verify >> $O/auto.jsonl 2>&1 || exit 1
done
python3 -c "
import json
for l in open('$O/auto.jsonl'):
    if l.startswith('{'):
        d = json.loads(l); print(d['mode'], d['bits'], d['bytes'] >> 20, d['ran'], d['gbps'], d['verified'])
"
