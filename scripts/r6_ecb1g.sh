set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6/ecb1g; mkdir -p $O
for b in 256M 512M 1G 2G 4G 8G; do
  timeout -k 10 60 ./bin/otbench --mode ecb --bits 128 --bytes $b --impl ttable --iters 20 --warmup 3 --clock >> $O/sweep_tt.jsonl 2>&1 || exit 1
  timeout -k 10 60 ./bin/otbench --mode ecb --bits 128 --bytes $b --iters 20 --warmup 3 >> $O/sweep_auto.jsonl 2>&1 || exit 1
done
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- ./bin/otbench --mode ecb --bits 128 --bytes 1G --iters 20 --warmup 3 > $O/kt.log 2>&1 || exit 1
