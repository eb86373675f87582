# Round 6: streaming-NT release build -- GPU suite, bench, then every routed
# mode against the pre-NT build.
set -e
D=gpurun_out/r6/f; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $D/all.log 2>&1
timeout -k 10 400 python bench.py > $D/bench.json 2> $D/bench.err
timeout -k 10 840 bash scripts/r6_final_nt_ab.sh > $D/final_nt_ab.txt 2>&1
timeout -k 10 400 bash scripts/r6_pmc_nt.sh > $D/pmc_nt.txt 2>&1
