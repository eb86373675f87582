#!/bin/bash
# Round 6: does the headline kernel wait on instruction fetch?  Its bulk
# form is ~105 KB of straight-line code (12.8k VALU, mostly 8-byte VOP3)
# per 2048-block task, more than the instruction cache it shares with the
# neighbouring CU.  Three PMC passes, each its own rocprofv3 run, AES-128
# CTR 16 GiB in place through the bitsliced bulk kernel.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r6/pmc_icache
mkdir -p $O
LIB=${LIB:-our_tree_amd/lib}
P1="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ"
P2="SQC_TC_INST_REQ SQC_TC_STALL SQC_ICACHE_BUSY_CYCLES SQC_ICACHE_INPUT_VALID_READYB"
P3="GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU"
TAG=${TAG:-base}
i=0
for C in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  LD_LIBRARY_PATH=$LIB timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d $O/$TAG-p$i -o run -- \
      ./bin/otbench --mode ctr --bits 128 --bytes 16G --inplace --iters 3 --warmup 1 > $O/$TAG-p$i.log 2>&1 ||
      { echo "FAILED pass $i"; tail -20 $O/$TAG-p$i.log; exit 1; }
done
csvs=$(find $O -path "*$TAG-p*" -name '*counter_collection.csv' | sort)
python3 tools/pmc_summary.py --kernel "k_aes_bs_t3<10, 0, 8, true, true>" $csvs > $O/$TAG.txt 2>&1 || true
cat $O/$TAG.txt
