# Round 6: the NT-default build -- GPU suite, bench, then NT beyond the headline.
set -e
D=gpurun_out/r6/e; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $D/all.log 2>&1
timeout -k 10 400 python bench.py > $D/bench.json 2> $D/bench.err
timeout -k 10 840 bash scripts/r6_ntall_ab.sh > $D/ntall_ab.txt 2>&1
