# Energy per VALU wave-instruction by instruction form: tools/ubench/valu_energy
# runs each form for ~8 s over the whole chip while amd-smi samples socket
# power and GFX clocks; summary = loaded power / instruction rate (nJ per
# wave-instruction, idle power included and reported separately).
#   gpurun --timeout 600 -- bash scripts/energy_probe.sh [ops]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
D=gpurun_out/energy
mkdir -p $D
ops=${1:-nop xor_vv and_vv bitop3_vvs bitop3_vvv bfi_vvv perm_vvv lshl_vi and_or_vvv ds_read_b32}
echo "== idle" >> $D/smi.txt
timeout 20 amd-smi metric -p -c -g 0 >> $D/smi.txt 2>&1
for op in $ops; do
    timeout -k 10 60 ./tools/ubench/valu_energy $op 8 >> $D/rates.jsonl 2>> $D/err.txt &
    P=$!
    sleep 3
    for i in 1 2 3; do
        echo "== $op" >> $D/smi.txt
        timeout 20 amd-smi metric -p -c -g 0 >> $D/smi.txt 2>&1
        sleep 1
    done
    wait $P || exit 1
done
python3 - <<'PY' | tee $D/summary.txt
import json, re
t = open("gpurun_out/energy/smi.txt").read()
pw = {}
clk = {}
for b in t.split("== ")[1:]:
    name = b.split("\n")[0].strip()
    m = re.search(r"SOCKET_POWER: (\S+) W", b)
    c = [int(x) for x in re.findall(r"GFX_\d:\n\s+CLK: (\d+) MHz", b)]
    if m: pw.setdefault(name, []).append(float(m.group(1)))
    if c: clk.setdefault(name, []).extend(c)
idle = min(pw.get("idle", [0]))
print(f"idle socket power {idle:.0f} W")
for l in open("gpurun_out/energy/rates.jsonl"):
    d = json.loads(l)
    op, r = d["op"], d["wave_instr_per_s"]
    w = sum(pw[op]) / len(pw[op])
    mhz = sum(clk[op]) / len(clk[op]) if op in clk else 0
    print(f"{op:12s} {r / 1e12:7.3f} T wave-instr/s  {w:6.0f} W  {mhz:5.0f} MHz  "
          f"{w / r * 1e9:7.3f} nJ/wave-instr  {(w - idle) / r * 1e9:7.3f} above idle")
PY
