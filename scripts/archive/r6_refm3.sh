set -e
D=gpurun_out/r6/refm3; mkdir -p $D
B="--steps 3 --warmup 1"
i=0
for opts in "" "--no-scatter" "--no-aes256 --no-other" "--no-stream"; do
  i=$((i+1)); echo "$opts" > $D/b$i.opts
  timeout -k 10 300 python bench.py $B $opts > $D/b$i.json 2>$D/b$i.err
done
HSA_ENABLE_SDMA=0 timeout -k 10 120 python -u tools/pipeline_state.py --only-big --recovery-s 4 --out $D/nosdma.jsonl > $D/nosdma.log 2>&1
