# Round 6 final build: the result logs again (HIP rows from the streaming-NT
# build), then a kernel trace of the whole bench -- does the profiler still
# crash at exit once the library returns its streams at interpreter exit?
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 bash scripts/r6_results.sh
D=gpurun_out/r6/final2; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o bench -- python3 bench.py --steps 5 --warmup 1 --no-power > $D/prof.log 2>&1
echo "profiled bench exit 0" >> $D/prof.log
