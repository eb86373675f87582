#!/bin/bash
# A/B of library builds on the box (run through gpurun):
#   bash scripts/ab_lib.sh REPS name=path/to/libotc.so ... -- [bench.py args]
# "default" means the in-tree our_tree_amd/lib/libotc.so.  The bench runs once
# per variant per rep, interleaved (v1 v2 v1 v2 ...), each under its own time
# limit; output lines prefixed with the variant name go to gpurun_out/ab.jsonl.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
reps=$1; shift
vars=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do vars+=("$1"); shift; done
[ "$1" = "--" ] && shift
mkdir -p gpurun_out
for r in $(seq 1 "$reps"); do
    for v in "${vars[@]}"; do
        name=${v%%=*}; lib=${v#*=}
        if [ "$lib" = "default" ]; then lib=""; fi
        line=$(OTC_LIB=$lib timeout -k 10 300 python bench.py "$@" 2>>gpurun_out/ab.err) || { echo "FAILED $name"; exit 1; }
        echo "{\"variant\": \"$name\", \"rep\": $r, \"bench\": $line}" | tee -a gpurun_out/ab.jsonl
    done
done
