# the ECB / CBC-dec split with its halves on CU-masked
# (dedicated-queue) streams vs HIP's pooled queues, on both runtimes.
C=""
for cfg in "--mode ecb --bits 256 --bytes 8G --iters 20" "--mode ecb --bits 256 --bytes 64G --inplace --iters 10" \
           "--mode cbc-dec --bits 256 --bytes 8G --iters 20"; do
    C="$C;$cfg --split-stats"
done
bash scripts/ab_runtime.sh r6/aux_queue_rt 2 "rt70 rt72" "${C#;}" base pooledaux
