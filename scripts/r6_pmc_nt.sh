#!/bin/bash
# Round 6: what the non-temporal bit changes in the headline kernel, by PMC.
# Two passes per library (prent = before NT, base = the release build): 8 SQ
# counters, then 4 TCC counters, each its own rocprofv3 run, AES-128 CTR 16
# GiB in place through the bitsliced bulk kernel.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r6/pmc_nt
mkdir -p $O variants/base
[ -f variants/base/libotc.so ] || cp our_tree_amd/lib/libotc.so variants/base/
SQ="GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_WR"
TCC="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
for v in prent base; do
  for pass in sq tcc; do
    if [ $pass = sq ]; then C=$SQ; else C=$TCC; fi
    LD_LIBRARY_PATH=variants/$v timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/$v-$pass -o run -- \
        ./bin/otbench --mode ctr --bits 128 --bytes 16G --inplace --iters 3 --warmup 1 > $O/$v-$pass.log 2>&1 ||
        { echo "FAILED $v $pass"; tail -20 $O/$v-$pass.log; exit 1; }
    csv=$(find $O/$v-$pass -name '*counter_collection.csv' | head -1)
    python3 tools/pmc_summary.py --kernel "k_aes_bs_t3<10, 0, 8, true, true>" "$csv" > $O/$v-$pass.txt 2>&1 || true
    echo "== $v $pass"; cat $O/$v-$pass.txt
  done
done
