#!/bin/bash
# Full GPU validation of the tree: smoke, pytest -m gpu, bench.py (1 GPU).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r5_full}; mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log; grep -c PASSED $O/pytest_gpu.log; grep -i "warning" $O/pytest_gpu.log | sort | uniq -c | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 3000 $O/bench.json
