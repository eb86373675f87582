#!/bin/bash
# Memory-pipeline counters: CBC-encrypt segments vs ECB (same bytes).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/profcbc
mkdir -p $OUT
for m in cbc-enc-seg ecb; do
  B="./bin/otbench --bytes 4G --iters 3 --warmup 1 --mode $m --impl ttable"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$m -o run -- $B > $OUT/kt_$m.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS TA_FLAT_WRITE_WAVEFRONTS TCP_TCC_READ_REQ TCC_HIT TCC_MISS --output-format csv -d $OUT/p1_$m -o run -- $B > $OUT/p1_$m.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_WRREQ TCC_EA0_WRREQ_64B TCC_EA0_RDREQ_DRAM SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d $OUT/p2_$m -o run -- $B > $OUT/p2_$m.log 2>&1 || exit 1
done
echo done
