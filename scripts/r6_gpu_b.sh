# Round 6: co-residency matrix (release + padded-descriptor build), the GPU
# suite minus the busy-process co-residency test, the bench, the census.
set -e
D=gpurun_out/r6/b; mkdir -p $D
timeout -k 10 240 python -u tools/coresidency_matrix.py --reps 2 --out $D/matrix.jsonl > $D/matrix.log 2>&1
OTC_LIB=variants/padclaim/libotc.so timeout -k 10 240 python -u tools/coresidency_matrix.py --reps 1 --out $D/matrix_padclaim.jsonl > $D/matrix_padclaim.log 2>&1
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread tests -m gpu --deselect tests/test_gpu_queues.py::test_split_halves_coresident_in_busy_process > $D/all.log 2>&1 || echo "pytest rc=$?" >> $D/all.log
timeout -k 10 400 python bench.py > $D/bench.json 2> $D/bench.err
timeout -k 10 300 python -u tools/pipeline_census.py --states torch,nccl,split,scatter,busy --out $D/census.jsonl > $D/census.log 2>&1
