# Round 6: the streaming-NT release build (bitsliced + coalesced T-table
# kernels) against the build before NT (prent), every routed mode incl. the
# segment chains that must stay on cached loads.
C="--mode ctr --bits 128 --bytes 64G --inplace --iters 10;--mode ctr --bits 256 --bytes 64G --inplace --iters 10"
C="$C;--mode ecb --bits 256 --bytes 64G --inplace --iters 10;--mode cbc-dec --bits 256 --bytes 8G --iters 20"
C="$C;--mode cfb-dec --bits 256 --bytes 8G --iters 20;--mode ecb-dec --bits 256 --bytes 8G --iters 20"
C="$C;--mode ctr --bits 128 --bytes 1G --iters 20;--mode ecb --bits 256 --bytes 1000M --iters 20"
C="$C;--mode cbc-enc-seg --bits 256 --bytes 8G --iters 10 --seg 4096;--mode cfb-enc-seg --bits 256 --bytes 1G --iters 10 --seg 4096"
C="$C;--mode cbc-dec-seg --bits 256 --bytes 8G --iters 20 --seg 4096"
bash scripts/ab_runtime.sh r6/final_nt_ab 2 "rt70" "$C" prent base
