# Round 6, final-build validation: GPU suite; the busy-process co-residency
# test on the padded-descriptor build (must FAIL: negative control); bench;
# the post-free copy probe; a kernel-trace profile of the bench's headline
# loop; the non-temporal A/B with power.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6/d1; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $D/all.log 2>&1
if OTC_LIB=variants/padclaim/libotc.so OTC_PRINT_UNITS=1 timeout -k 10 300 python -u -m pytest -v -s --timeout 120 \
     --timeout-method thread tests/test_gpu_queues.py -m gpu -k coresident > $D/queues_padclaim.log 2>&1; then
  echo "NEGATIVE CONTROL PASSED (unexpected)" >> $D/queues_padclaim.log
else
  echo "negative control failed as expected (rc=$?)" >> $D/queues_padclaim.log
fi
timeout -k 10 400 python bench.py > $D/bench.json 2> $D/bench.err
timeout -k 10 120 python -u tools/free_wipe_probe.py --gib 64 --seconds 8 --out $D/free_wipe.jsonl > $D/free_wipe.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o bench -- python3 bench.py --steps 5 --warmup 1 --no-stream --no-scatter --no-other-impl --no-aes256 --no-refmethod --no-power > $D/prof.log 2>&1
timeout -k 10 600 bash scripts/r6_nt_ab.sh > $D/nt_ab.txt 2>&1
