#!/bin/bash
# Socket power, clocks and PPT-limit residency over the timed loop of each
# AES-256 ECB / decrypt / CBC kernel (and the CTR kernels for reference), all
# verified; then one PMC pass over the T-table ECB encrypt / decrypt kernels.
# Round-3 review item 1(a).   gpurun --timeout 900 -- bash scripts/r4_power.sh NAME
# -> gpurun_out/NAME/power.jsonl (otbench JSON + "power" + joules_per_gb)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r4_power}
mkdir -p $O
run() { # label, otbench args (each loop ~8 s)
    local label=$1
    shift
    timeout -k 10 150 python3 tools/power_run.py --label "$label" -- ./bin/otbench "$@" --verify --mark \
        >> $O/power.jsonl 2>> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
    python3 - "$O/power.jsonl" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
p = d["power"]
print(f'{d["label"]:18s} {d["gbps"]:8.1f} GB/s  verified={d["verified"]}  {p.get("avg_socket_w")} W  '
      f'{d.get("joules_per_gb")} J/GB  PPT {p.get("ppt_residency")}  gfx {p.get("gfxclk_mhz_min")}-{p.get("gfxclk_mhz_max")} MHz')
PY
}
ONLY=${ONLY:-all}
if [ "$ONLY" = all ] || [ "$ONLY" = ecb ]; then
run tt-ecb256-4g    --mode ecb --bits 256 --bytes 4G --inplace --impl ttable --iters 1900 --warmup 20
run bs-ecb256-4g    --mode ecb --bits 256 --bytes 4G --inplace --impl bitslice --iters 1900 --warmup 20
run tt-ecb256-64g   --mode ecb --bits 256 --bytes 64G --inplace --impl ttable --iters 120 --warmup 2
run bs-ecb256-64g   --mode ecb --bits 256 --bytes 64G --inplace --impl bitslice --iters 120 --warmup 2
run tt-ecbdec256-4g --mode ecb-dec --bits 256 --bytes 4G --inplace --iters 1900 --warmup 20
run tt-ecbdec256-64g --mode ecb-dec --bits 256 --bytes 64G --inplace --iters 120 --warmup 2
run tt-cbcdec256-4g --mode cbc-dec --bits 256 --bytes 4G --iters 1900 --warmup 20
run tt-cbcdec256-32g --mode cbc-dec --bits 256 --bytes 32G --iters 240 --warmup 2
fi
if [ "$ONLY" = all ] || [ "$ONLY" = ctr ]; then
run bs-ctr128-64g   --mode ctr --bits 128 --bytes 64G --inplace --impl bitslice --iters 200 --warmup 2
run tt-ctr128-64g   --mode ctr --bits 128 --bytes 64G --inplace --impl ttable --iters 180 --warmup 2
run bs-ctr256-64g   --mode ctr --bits 256 --bytes 64G --inplace --impl bitslice --iters 150 --warmup 2
fi
if [ "$ONLY" = all ] || [ "$ONLY" = pmc ]; then
C="GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY"
for m in ecb ecb-dec; do
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$m -o run -- \
        ./bin/otbench --mode $m --bits 256 --bytes 4G --impl ttable --inplace --iters 3 --warmup 1 > $O/pmc_$m.log 2>&1 ||
        { tail -20 $O/pmc_$m.log; exit 1; }
    csv=$(find $O/pmc_$m -name '*counter_collection.csv' | head -1)
    k=k_aes_enc_tt; [ $m = ecb-dec ] && k=k_aes_dec_tt
    python3 tools/pmc_summary.py --kernel "$k" "$csv" > $O/pmc_${m}256_tt.txt && cat $O/pmc_${m}256_tt.txt
done
fi
