set -e
mkdir -p gpurun_out/r6/refm2
B="--steps 3 --warmup 1 --no-other --no-aes256 --no-stream"
i=0
for opts in "--no-power --no-clock" "--no-power" "--no-clock" "--gib 4" ""; do
  i=$((i+1))
  echo "$opts" > gpurun_out/r6/refm2/b$i.opts
  timeout -k 10 300 python bench.py $B $opts > gpurun_out/r6/refm2/b$i.json 2>gpurun_out/r6/refm2/b$i.err
done
