# Round 6: the serving path (ops.CtrBatch, one launch over many messages with
# their own keys / counters) with and without the non-temporal bit on the
# message loads / stores, interleaved, 3 reps, four batch shapes.
set -e
D=gpurun_out/r6/batch_nt; mkdir -p $D
for r in 1 2 3; do
  for v in base batchnt; do
    L=our_tree_amd/lib/libotc.so; [ $v = batchnt ] && L=variants/batchnt/libotc.so
    for shape in "--msgs 16384 --size 4096 --keys 256" "--msgs 65536 --size 1504 --keys 1024" \
                 "--msgs 262144 --size 4096 --keys 256" "--msgs 1024 --size 1048576 --keys 64"; do
      echo "{\"variant\": \"$v\", \"rep\": $r, \"shape\": \"$shape\"}" >> $D/ab.jsonl
      OTC_LIB=$L timeout -k 10 200 python benchmarks/batch_ctr.py $shape --no-eager --iters 20 >> $D/ab.jsonl 2>> $D/err.txt
    done
  done
done
