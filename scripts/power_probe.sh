# Socket power and GFX clocks (amd-smi, every 2 s) while bench.py runs the
# headline CTR step for ~9 s with each kernel, then energy per byte
# (average loaded socket power / GB/s = nJ per byte = J per GB); writes
# gpurun_out/power/.   gpurun --timeout 600 -- bash scripts/power_probe.sh [impls]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/power
impls=${1:-ttable bitslice}
for impl in $impls; do
    timeout -k 10 300 python bench.py --steps 200 --warmup 3 --impl $impl --no-aes256 --no-scatter --no-stream \
        --no-other-impl --no-clock > gpurun_out/power/bench_$impl.json 2> gpurun_out/power/bench_$impl.err &
    P=$!
    for i in $(seq 1 8); do
        sleep 2; echo "== $(date +%T) $impl" >> gpurun_out/power/smi.txt
        timeout 20 amd-smi metric -p -c -t -v -g 0 >> gpurun_out/power/smi.txt 2>&1
    done
    wait $P || exit 1
done
python3 - <<'PY' | tee gpurun_out/power/summary.txt
import json, re
t = open("gpurun_out/power/smi.txt").read()
loaded = {}
for b in t.split("== ")[1:]:
    head = b.split("\n")[0]
    pw = re.search(r"SOCKET_POWER: (\S+) W", b)
    clks = [int(x) for x in re.findall(r"GFX_\d:\n\s+CLK: (\d+) MHz", b)]
    print(head, pw.group(1) + " W" if pw else "-", "gfx MHz %d-%d" % (min(clks), max(clks)) if clks else "-")
    if pw:
        loaded.setdefault(head.split()[-1], []).append(float(pw.group(1)))
for impl, ws in loaded.items():
    gbps = json.load(open(f"gpurun_out/power/bench_{impl}.json"))["value"]
    ws = [x for x in ws if x >= 0.9 * max(ws)]  # steady state: drop the ramp and idle samples
    w = sum(ws) / len(ws)
    print(f"{impl}: {gbps:.1f} GB/s at {w:.0f} W loaded socket power = {w / gbps:.3f} J/GB (nJ/B)")
PY
