set -e
D=gpurun_out/r6/state2; mkdir -p $D
timeout -k 10 120 python -u tools/pipeline_state.py --only-big --recovery-s 6 --out $D/a_default.jsonl > $D/a.log 2>&1
timeout -k 10 120 python -u tools/pipeline_state.py --only-big --no-kernel --recovery-s 3 --out $D/b_nokernel.jsonl > $D/b.log 2>&1
timeout -k 10 120 python -u tools/pipeline_state.py --only-big --keep-cache --recovery-s 3 --out $D/c_keepcache.jsonl > $D/c.log 2>&1
timeout -k 10 120 python -u tools/pipeline_state.py --only-big --gib 8 --recovery-s 3 --out $D/d_8g.jsonl > $D/d.log 2>&1
