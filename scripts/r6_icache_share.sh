#!/bin/bash
# Round 6: is the headline kernel sensitive to instruction-cache sharing?
# The full chip (power-capped, ~1.75 GHz) against CUs 0-127 only (HSA_CU_MASK
# restricts every queue of the process; half the power, so ~2.39 GHz): if
# memory or fetch latency limited issue, VALU per clock per active CU would
# fall at the higher clock.  (A mask of every other CU, to halve instruction-
# cache sharing, was not applied by the runtime: a 128-entry CU list.)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r6/icache_share
mkdir -p $O
P1="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ"
P3="GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU"
for cfg in all half; do
  case $cfg in
    all) M="" ;;
    half) M="0:0-127" ;;
  esac
  i=0
  for C in "$P1" "$P3"; do
    i=$((i + 1))
    HSA_CU_MASK=$M timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d $O/$cfg-p$i -o run -- \
        ./bin/otbench --mode ctr --bits 128 --bytes 8G --inplace --iters 3 --warmup 1 > $O/$cfg-p$i.log 2>&1 ||
        { echo "FAILED $cfg pass $i"; tail -20 $O/$cfg-p$i.log; exit 1; }
  done
  csvs=$(find $O -path "*/$cfg-p*" -name '*counter_collection.csv' | sort)
  python3 tools/pmc_summary.py --kernel "k_aes_bs_t3<10, 0, 8, true, true>" $csvs > $O/$cfg.txt 2>&1 || true
  echo "== $cfg"; cat $O/$cfg.txt
done
