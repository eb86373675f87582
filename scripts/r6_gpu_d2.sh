# Round 6: result logs in the reference formats, then the split's auxiliary
# streams on dedicated vs pooled queues on both runtimes.
set -e
timeout -k 10 1000 bash scripts/r6_results.sh
timeout -k 10 600 bash scripts/r6_aux_queue_rt.sh > gpurun_out/r6/aux_queue_rt.txt 2>&1
