#!/bin/bash
# Round 6 last build: GPU suite, smoke(), the driver bench twice, a kernel
# trace of the whole bench, and BASELINE configs 4 / 5 at full size on one GPU.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6/${OUT:-final4}; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $D/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
timeout -k 10 400 python bench.py > $D/bench.json 2> $D/bench.err
timeout -k 10 400 python bench.py > $D/bench2.json 2> $D/bench2.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o bench -- python3 bench.py --steps 5 --warmup 1 --no-power > $D/prof.log 2>&1
timeout -k 10 300 python benchmarks/cbc_scatter.py --gib-per-gpu 256 > $D/config4.json 2> $D/config4.err
timeout -k 10 400 python benchmarks/stream_ctr.py --total-gib 1024 > $D/config5.json 2> $D/config5.err
