# Round 6: auxiliary streams warmed at creation -- the first split call of a
# fresh process must co-run (queue test alone, then the matrix), then the
# suite and the bench.
set -e
D=gpurun_out/r6/h; mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_queues.py -m gpu > $D/queues.log 2>&1
timeout -k 10 240 python -u tools/coresidency_matrix.py --reps 1 --out $D/matrix.jsonl > $D/matrix.log 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $D/all.log 2>&1
timeout -k 10 400 python bench.py > $D/bench.json 2> $D/bench.err
