#!/bin/bash
# (evidence script: the knob it varied was removed from the source after the A/B; see docs/PERF.md round 5)
# RC4 PRGA byte-index addressing: 3 VALU (base, OTC_RC4_ADDR3=1) vs 5 (rc4old).
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r5_rc4_ab}; mkdir -p $O
for r in 1 2 3; do for cfg in "131072 8K" "163840 8K" "1M 1K" "65536 64K"; do for v in base rc4old; do
    set -- $cfg
    LD_LIBRARY_PATH=variants/$v timeout -k 10 60 ./bin/otbench --mode rc4 --streams $1 --len $2 --iters 10 --verify > $O/last.json 2>> $O/err.txt || { echo "FAILED $v $cfg"; tail -5 $O/err.txt; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/last.json')); d['variant']='$v'; print(json.dumps(d))" | tee -a $O/ab.jsonl | cut -c1-60,100-200
done; done; done
