set -e
mkdir -p gpurun_out/r6/census2
timeout -k 10 300 python -u tools/pipeline_census.py --states torch,scatter --realloc --out gpurun_out/r6/census2/a.jsonl > gpurun_out/r6/census2/a.log 2>&1
timeout -k 10 300 python -u tools/pipeline_census.py --states nccl,scatter --out gpurun_out/r6/census2/b.jsonl > gpurun_out/r6/census2/b.log 2>&1
