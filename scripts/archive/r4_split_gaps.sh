#!/bin/bash
# Per-call timeline of small split calls (kernel trace): where do ~150 us go?
# SIZE=256M for a mid-size call (default 64M)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r4_split_gaps}
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d $O/db -o run -- ./bin/otbench --mode ecb --bits 256 \
    --bytes ${SIZE:-64M} --inplace --impl split --iters 20 --warmup 2 > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
db=$(find $O/db -name '*.db' | head -1)
python3 - "$db" > $O/gaps.txt <<'PY'
import sqlite3, sys
db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, start, end, queue_id from kernels order by start").fetchall()
t0 = rows[0][1]
for n, s, e, q in rows[-60:]:
    print(f"{(s - t0) / 1e3:12.1f} {(e - s) / 1e3:9.1f} q{q} {n[:90]}")
PY
tail -60 $O/gaps.txt
python3 tools/split_timeline.py "$db" --label "ecb-256 ${SIZE:-64M}" > $O/timeline.txt && tail -25 $O/timeline.txt
