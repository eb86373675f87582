#!/bin/bash
# PMC of the persistent T-table claim kernels alone: segment encryption
# (CBC-enc-seg-256, 4 KiB segments, 4 GiB in place -> k_aes_seg_enc_tt_claim)
# against ECB-256 (1536 MiB, auto -> k_aes_ecb_tt_claim alone).  One counter
# group per pass.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r5_pmc_ttclaim}; mkdir -p $O
for cfg in "seg:--mode cbc-enc-seg --bits 256 --seg 4096 --bytes 4G --inplace:seg_enc_tt_claim" "ecb:--mode ecb --bits 256 --bytes 1536M --inplace:ecb_tt_claim"; do
    IFS=: read -r name args kern <<< "$cfg"
    i=0
    for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" \
                "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
                "FETCH_SIZE" "WRITE_SIZE"; do
        i=$((i+1))
        timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-include-regex "$kern" -d $O/p_${name}_$i -o p -- ./bin/otbench $args --iters 3 --warmup 1 > $O/run_${name}_$i.txt 2>&1 || { echo "pass $name $i failed"; tail -5 $O/run_${name}_$i.txt; exit 1; }
    done
    bytes=$(python3 -c "import json; print([json.loads(l) for l in open('$O/run_${name}_1.txt') if l.startswith('{')][-1]['bytes'])")
    python3 tools/rocpd_pmc.py --kernel $kern --bytes $bytes $(find $O -path "*p_${name}_*" -name "*.db" | sort) > $O/pmc_$name.txt 2>&1
    cat $O/pmc_$name.txt
done
