# Round 6: the bs8-free build -- GPU suite, bench, then the CTR split A/B on
# both runtimes.
set -e
D=gpurun_out/r6/c; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $D/all.log 2>&1
timeout -k 10 400 python bench.py > $D/bench.json 2> $D/bench.err
timeout -k 10 900 bash scripts/r6_ctr_split_rt.sh > $D/ctr_split_rt.txt 2>&1
