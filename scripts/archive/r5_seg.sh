#!/bin/bash
# Round 5: the chained segment-encryption split (T-table + row-sliced bs8).
# 1) the new GPU tests, 2) otbench ttable / bitslice / split for CBC / CFB
# encryption of 4 KiB and 512 B segments, AES-256 and AES-128, verified, with
# socket power (tools/power_run.py) -> gpurun_out/$OUT/ab.jsonl
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=${1:-r5_seg}; SIZES=${2:-"4G"}; ITERS=${3:-60}
O=gpurun_out/$OUT
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py \
    -k "segment_encrypt_split or split_bitsliced_alone or cbc_segments or cfb128_segments or segment_decrypt_split" \
    > $O/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
fi
for sz in $SIZES; do for bits in 256 128; do for seg in 4096 512; do for mode in cbc-enc-seg cfb-enc-seg; do
  [ "$bits" = 128 ] && [ "$mode" = cfb-enc-seg ] && continue
  for impl in ttable bitslice split; do
    timeout -k 10 120 python3 tools/power_run.py --label $impl/$seg -- ./bin/otbench --mode $mode --bits $bits \
        --bytes $sz --seg $seg --inplace --iters $ITERS --warmup 3 --impl $impl --verify --mark \
        >> $O/ab.jsonl 2>> $O/err.txt || { echo "FAILED $mode $bits $seg $impl"; tail -5 $O/err.txt; exit 1; }
    python3 - "$O/ab.jsonl" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
p = d["power"]
print(f'{d["label"]:13s} ran={d["ran"]:8s} {d["mode"]:11s} {d["bits"]} {d["bytes"] >> 20:6d}M {d["gbps"]:8.1f} GB/s v={d["verified"]} '
      f'{p.get("avg_socket_w")} W {d.get("joules_per_gb")} J/GB PPT {p.get("ppt_residency")} gfx {p.get("gfxclk_mhz_mean")} MHz', flush=True)
PY
  done
done; done; done; done
