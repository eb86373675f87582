# Round 6 validation: queue/co-residency tests (+ padded-descriptor negative
# control), the whole GPU suite, the driver bench, and the pipeline census.
set -e
D=gpurun_out/r6/a; mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_queues.py -m gpu > $D/queues.log 2>&1
if [ -f variants/padclaim/libotc.so ]; then
  OTC_LIB=variants/padclaim/libotc.so OTC_PRINT_UNITS=1 timeout -k 10 300 python -u -m pytest -v -s --timeout 120 --timeout-method thread tests/test_gpu_queues.py -m gpu -k coresident > $D/queues_padclaim.log 2>&1 || echo "padclaim pytest rc=$?" >> $D/queues_padclaim.log
fi
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $D/all.log 2>&1
timeout -k 10 400 python bench.py > $D/bench.json 2> $D/bench.err
timeout -k 10 300 python -u tools/pipeline_census.py --states torch,nccl,split,scatter,busy --out $D/census.jsonl > $D/census.log 2>&1
