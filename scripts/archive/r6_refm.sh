set -e
mkdir -p gpurun_out/r6/refm
timeout -k 10 200 python -c "
import sys,json; sys.path.insert(0,'.')
import torch; torch.cuda.set_device(0)
from our_tree_amd.utils import refmethod
r=refmethod.ecb256_three_ways(device=0); print(json.dumps({'run':'standalone',**r}))
" > gpurun_out/r6/refm/standalone.json 2>gpurun_out/r6/refm/standalone.err
for opts in "--no-other --no-aes256 --no-stream --no-scatter" "--no-other --no-aes256 --no-stream" "--no-other --no-aes256 --no-scatter" "--no-stream --no-scatter"; do
  tag=$(echo $opts | tr -d ' -')
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 $opts > gpurun_out/r6/refm/b_$tag.json 2>gpurun_out/r6/refm/b_$tag.err
done
