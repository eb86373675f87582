# Round 6: does the split's 2 GiB threshold still hold on the streaming-NT
# build?  auto (= the persistent T-table claim kernel below 2 GiB) vs an
# explicit split, ECB / CBC-dec, AES-128 / 256, 1 and 1.5 GiB, 3 reps.
C=""
for m in ecb cbc-dec; do for b in 128 256; do for sz in 1G 1536M; do
  for i in auto split; do C="$C;--mode $m --bits $b --bytes $sz --iters 50 --impl $i --split-stats"; done
done; done; done
bash scripts/ab_runtime.sh r6/split_threshold 3 "rt70" "${C#;}" base
