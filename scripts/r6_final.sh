# Round 6 final build: GPU suite, smoke(), the driver bench twice, and a
# kernel-trace profile of the whole bench (every extra pass).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6/${OUT:-final}; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $D/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
timeout -k 10 400 python bench.py > $D/bench.json 2> $D/bench.err
timeout -k 10 400 python bench.py > $D/bench2.json 2> $D/bench2.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o bench -- python3 bench.py --steps 5 --warmup 1 --no-power > $D/prof.log 2>&1
