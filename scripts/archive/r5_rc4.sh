#!/bin/bash
# RC4 many-stream kernel: what bounds it.
#  1. occupancy scaling: GB/s against resident streams per CU (8 KiB streams;
#     LDS holds at most 10 waves = 640 streams per CU)
#  2. PMC at 131072 x 8 KiB and 1M x 1 KiB, one counter group per pass
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r5_rc4}; mkdir -p $O
for s in 16384 32768 65536 98304 131072 163840 196608 327680; do
    timeout -k 10 60 ./bin/otbench --mode rc4 --streams $s --len 8K --iters 10 --verify >> $O/scaling.jsonl 2>> $O/err.txt || { echo "scaling $s failed"; tail -5 $O/err.txt; exit 1; }
    tail -1 $O/scaling.jsonl
done
timeout -k 10 60 ./bin/otbench --mode rc4 --streams 1M --len 1K --iters 10 --verify >> $O/scaling.jsonl 2>> $O/err.txt || exit 1
tail -1 $O/scaling.jsonl
for cfg in "131072 8K" "1M 1K"; do
    set -- $cfg
    n=${1}x$2; i=0
    for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES" \
                "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
                "SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_IFETCH SQ_WAVES"; do
        i=$((i+1))
        timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-include-regex "k_rc4_kernel" -d $O/p_${n}_$i -o p -- \
            ./bin/otbench --mode rc4 --streams $1 --len $2 --iters 3 --warmup 1 > $O/run_${n}_$i.txt 2>&1 || { echo "pass $n $i failed"; tail -5 $O/run_${n}_$i.txt; exit 1; }
    done
    python3 tools/rocpd_pmc.py --kernel k_rc4_kernel $(find $O -path "*p_${n}_*" -name "*.db" | sort) > $O/pmc_$n.txt 2>&1
    cat $O/pmc_$n.txt
done
