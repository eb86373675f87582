#!/bin/bash
# Re-entry validation: GPU tests, smoke, headline bench.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r1e
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1; rc=$?; tail -2 $OUT/bench.log; exit $rc
