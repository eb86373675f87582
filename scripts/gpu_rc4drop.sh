#!/bin/bash
# RC4-drop768 with 1 KiB streams: aligned drop loop (default) vs generic loops
# (OTC_RC4_ALIGNED=0), after the RC4 tests.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/rc4drop
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "rc4 or arc4" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cat > $OUT/t.py <<'PY'
import json, os, sys, time, torch
sys.path.insert(0, os.getcwd())
from our_tree_amd import ops
ns, L, drop = 1 << 20, 1024, 768
keys = torch.randint(0, 256, (ns, 16), dtype=torch.uint8, device="cuda")
ops.rc4_multi(keys, L, drop=drop); torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(5): ops.rc4_multi(keys, L, drop=drop)
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / 5
print(json.dumps({"streams": ns, "len": L, "drop": drop, "aligned": os.environ.get("OTC_RC4_ALIGNED", "default"),
                  "ms": round(dt * 1e3, 3), "gbps_output": round(ns * L / dt / 1e9, 2)}))
PY
for rep in 1 2; do
for al in 0 2; do
  OTC_RC4_ALIGNED=$al timeout -k 10 120 python $OUT/t.py >> $OUT/drop.jsonl 2>> $OUT/err.log || exit 1
done
done
cat $OUT/drop.jsonl
