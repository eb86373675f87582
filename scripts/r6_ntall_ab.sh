# Round 6: non-temporal streaming beyond the headline kernel.  prent = the
# build before NT (release of commit bdeacdc), base = NT in the bitsliced
# kernel (CTR loads, every bitsliced store -- the new default), ntall = also
# the T-table kernels' block loads / stores and the bitsliced ECB-plane loads.
C="--mode ctr --bits 128 --bytes 64G --inplace --iters 10"
C="$C;--mode ecb --bits 256 --bytes 64G --inplace --iters 10;--mode ecb --bits 256 --bytes 8G --iters 20"
C="$C;--mode cbc-dec --bits 256 --bytes 8G --iters 20;--mode cfb-dec --bits 256 --bytes 8G --iters 20"
C="$C;--mode ecb-dec --bits 256 --bytes 8G --iters 20;--mode ctr --bits 128 --bytes 16G --iters 20 --impl ttable"
C="$C;--mode cbc-enc-seg --bits 256 --bytes 8G --iters 10 --seg 4096"
bash scripts/ab_runtime.sh r6/ntall_ab 2 "rt70" "$C" prent base ntall
