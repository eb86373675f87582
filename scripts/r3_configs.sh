#!/bin/bash
# Round-3 evidence run (through gpurun): configs 4 and 5 at full size through
# the --gpus self-launch, AES-256 ECB T-table vs bitsliced at 64 GiB, a PMC
# pass of the bulk bitsliced CTR kernel, and the power probe (J/GB).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r3cfg; mkdir -p $O
timeout -k 10 300 python benchmarks/cbc_scatter.py --gpus 1 --gib-per-gpu 256 > $O/cfg4_cbc256_enc_256g.json 2> $O/cfg4_enc.err || { tail -5 $O/cfg4_enc.err; exit 1; }
cat $O/cfg4_cbc256_enc_256g.json
timeout -k 10 300 python benchmarks/cbc_scatter.py --gpus 1 --gib-per-gpu 256 --decrypt > $O/cfg4_cbc256_dec_256g.json 2> $O/cfg4_dec.err || { tail -5 $O/cfg4_dec.err; exit 1; }
cat $O/cfg4_cbc256_dec_256g.json
timeout -k 10 300 python benchmarks/stream_ctr.py --gpus 1 --total-gib 1024 > $O/cfg5_ctr128_stream_1t.json 2> $O/cfg5.err || { tail -5 $O/cfg5.err; exit 1; }
cat $O/cfg5_ctr128_stream_1t.json
for i in ttable bitslice; do for r in 1 2; do
    timeout -k 10 180 ./bin/otbench --mode ecb --bits 256 --bytes 64G --inplace --iters 5 --warmup 1 --impl $i --clock >> $O/ecb256_64g.jsonl || exit 1
done; done
cat $O/ecb256_64g.jsonl
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/pmc -o run -- ./bin/otbench --mode ctr --impl bitslice --bytes 4G --iters 5 --warmup 1 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
bash scripts/power_probe.sh "ttable bitslice"
