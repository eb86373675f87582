# Socket power and GFX clocks (amd-smi, every 2 s) while bench.py runs the
# headline CTR step for ~9 s with each kernel; writes gpurun_out/power/.
#   gpurun --timeout 600 -- bash scripts/power_probe.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/power
for impl in ttable bitslice; do
    timeout -k 10 300 python bench.py --steps 200 --warmup 3 --impl $impl --no-aes256 --no-scatter --no-bitslice \
        --no-clock > gpurun_out/power/bench_$impl.json 2> gpurun_out/power/bench_$impl.err &
    P=$!
    for i in $(seq 1 8); do
        sleep 2; echo "== $(date +%T) $impl" >> gpurun_out/power/smi.txt
        timeout 20 amd-smi metric -p -c -t -v -g 0 >> gpurun_out/power/smi.txt 2>&1
    done
    wait $P || exit 1
done
python3 - <<'PY'
import re
t = open("gpurun_out/power/smi.txt").read()
for b in t.split("== ")[1:]:
    head = b.split("\n")[0]
    pw = re.search(r"SOCKET_POWER: (\S+) W", b)
    clks = [int(x) for x in re.findall(r"GFX_\d:\n\s+CLK: (\d+) MHz", b)]
    print(head, pw.group(1) + " W" if pw else "-", "gfx MHz %d-%d" % (min(clks), max(clks)) if clks else "-")
PY
