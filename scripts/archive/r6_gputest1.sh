set -e
D=gpurun_out/r6/t1; mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_queues.py -m gpu > $D/queues.log 2>&1
OTC_LIB=variants/padclaim/libotc.so OTC_PRINT_UNITS=1 timeout -k 10 300 python -u -m pytest -v -s --timeout 120 --timeout-method thread tests/test_gpu_queues.py -m gpu -k coresident > $D/queues_padclaim.log 2>&1 || echo "padclaim rc=$?" >> $D/queues_padclaim.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $D/all.log 2>&1
timeout -k 10 400 python bench.py > $D/bench.json 2> $D/bench.err
