# the CTR split against the bitsliced kernel, on both
# HIP runtimes, AES-128 / 256 at 64 GiB in place and 16 GiB.
C=""
for cfg in "--bits 128 --bytes 64G --inplace --iters 10" "--bits 256 --bytes 64G --inplace --iters 10" \
           "--bits 128 --bytes 16G --iters 20" "--bits 256 --bytes 16G --iters 20"; do
    for i in bitslice split; do C="$C;--mode ctr $cfg --impl $i --split-stats"; done
done
bash scripts/ab_runtime.sh r6/ctr_split_rt 2 "rt70 rt72" "${C#;}" base
