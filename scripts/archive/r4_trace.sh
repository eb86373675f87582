#!/bin/bash
# Kernel + copy trace of the single-process RCCL scatter/gather job
# (otc_multi_run strategy 1, a 1-rank ncclCommInitAll on one GPU), and which
# of its phases overlapped (tools/overlap_summary.py).  Round-3 review item 6.
#   gpurun --timeout 600 -- bash scripts/r4_trace.sh NAME
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r4_trace}
mkdir -p $O
for m in ctr cbc-dec; do
    timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/db_$m -o run -- \
        ./bin/otbench --mode $m --bits 256 --e2e --strategy rccl --gpus 1 --bytes 4G --chunk 256M --warmup 1 --verify \
        > $O/run_$m.log 2>&1 || { tail -20 $O/run_$m.log; exit 1; }
    db=$(find $O/db_$m -name '*.db' | head -1)
    python3 - "$db" > $O/schema_$m.txt <<'PY'
import sqlite3, sys
db = sqlite3.connect(f"file:{sys.argv[1]}?mode=ro", uri=True)
for (n,) in db.execute("select name from sqlite_master where type in ('table','view') order by name"):
    if n in ("kernels", "memory_copies"):
        print(n, [c[1] for c in db.execute(f"pragma table_info({n})")])
PY
    python3 tools/overlap_summary.py "$db" > $O/overlap_$m.txt; cat $O/schema_$m.txt $O/overlap_$m.txt; tail -1 $O/run_$m.log
done
