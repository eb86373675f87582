#!/bin/bash
# Round 6: ops.CtrBatch with claimed tile runs for large batches (release,
# from 65536 tiles) vs the static split over the waves
# (OTC_BATCH_CLAIM_MIN_TILES=10^12), 3 interleaved reps, four shapes; the GPU
# batch tests first.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
D=gpurun_out/r6/batch_claim; mkdir -p $D
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "batch" > $D/pytest.log 2>&1 ||
    { tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for r in 1 2 3; do
  for v in static claimed; do
    if [ $v = static ]; then export OTC_BATCH_CLAIM_MIN_TILES=1000000000000; else unset OTC_BATCH_CLAIM_MIN_TILES; fi
    for shape in "--msgs 262144 --size 4096 --keys 256" "--msgs 1024 --size 1048576 --keys 64" \
                 "--msgs 4096 --size 1048576 --keys 64" "--msgs 16384 --size 4096 --keys 256"; do
      echo "{\"variant\": \"$v\", \"rep\": $r, \"shape\": \"$shape\"}" >> $D/ab.jsonl
      timeout -k 10 200 python3 benchmarks/batch_ctr.py $shape --no-eager --iters 20 >> $D/ab.jsonl 2>> $D/err.txt || exit 1
    done
  done
done
unset OTC_BATCH_CLAIM_MIN_TILES
python3 - <<'PY'
import json
cur = None
for l in open("gpurun_out/r6/batch_claim/ab.jsonl"):
    d = json.loads(l)
    if "variant" in d:
        cur = d
        continue
    print(cur["variant"], cur["rep"], cur["shape"], {k: d[k]["gbps"] for k in ("batch", "batch_packed") if k in d},
          d.get("verified_sample"))
PY
