#!/bin/bash
# PMC of the bs8 kernel alone (impl bitslice), CBC-enc-seg AES-256 4 GiB,
# 4 KiB segments: VALU rate, waits, HBM bytes.  One counter group per pass.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r5_pmc_bs8}; mkdir -p $O
LIB=${2:-}
ARGS="--mode cbc-enc-seg --bits 256 --bytes 4G --seg 4096 --inplace --iters 5 --warmup 1 --impl ${3:-bitslice}"
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
            "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  LD_LIBRARY_PATH=$LIB timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-include-regex "bs8|seg_enc" -d $O/p$i -o p -- ./bin/otbench $ARGS > $O/run$i.txt 2>&1 || { echo "pass $i failed"; tail -5 $O/run$i.txt; exit 1; }
done
python3 tools/pmc_summary.py --kernel ${4:-bs8} $(find $O -name "*counter_collection.csv" | sort) > $O/summary.txt 2>&1; head -60 $O/summary.txt
