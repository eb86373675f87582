# one energy reduction on the headline kernel, A/B with
# power -- non-temporal plaintext loads / ciphertext stores (OTC_BS_NT=1)
# against the release build, AES-128 / 256 CTR at 64 GiB in place, on the
# runtime bench.py binds (rt70).
C="--mode ctr --bits 128 --bytes 64G --inplace --iters 20 --clock;--mode ctr --bits 256 --bytes 64G --inplace --iters 20 --clock"
bash scripts/ab_runtime.sh r6/nt_ab 3 "rt70" "$C" base nt
