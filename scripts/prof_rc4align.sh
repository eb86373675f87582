#!/bin/bash
# RC4 i-aligned PRGA vs generic: SQ counters (one pass each), then a
# kernel-trace + stats run of the headline bench on the current build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/profrc4
mkdir -p $OUT
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
for al in 0 1; do
  OTC_RC4_ALIGNED=$al timeout -s KILL 90 rocprofv3 --pmc $C -d $OUT/al$al -o rc4 -- ./bin/otbench --mode rc4 --streams 131072 --len 8K --iters 4 --warmup 1 > $OUT/al$al.log 2>&1 || { tail -20 $OUT/al$al.log; exit 1; }
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/bench -o bench -- python3 bench.py --steps 5 --warmup 2 --no-clock > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
find $OUT -name "*.csv" -o -name "*.db" | head -20
