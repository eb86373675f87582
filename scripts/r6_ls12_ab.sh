# Round 6: 12 LDS-staged plaintext slots per wave (48 KiB per workgroup, 3
# workgroups = 144 KiB per CU) vs 8, with the streaming-NT release build.
C="--mode ctr --bits 128 --bytes 64G --inplace --iters 10;--mode ctr --bits 256 --bytes 64G --inplace --iters 10"
bash scripts/ab_runtime.sh r6/ls12_ab 3 "rt70" "$C" base ls12
