#!/bin/bash
# GB/s and J/GB of every mode x key size with impl=auto (the final build),
# verified, energy over each timed loop (tools/power_run.py), 4 GiB resident
# (in place where the mode allows), ~3 s per loop.
#   gpurun --timeout 900 -- bash scripts/r4_energy_table.sh NAME
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r4_energy_table}
mkdir -p $O
for m in ctr ecb ecb-dec cbc-dec cfb-dec cbc-enc-seg cfb-enc-seg cbc-dec-seg cfb-dec-seg; do
    for b in 128 192 256; do
        ip=--inplace
        case $m in cbc-dec|cfb-dec|cbc-dec-seg|cfb-dec-seg) ip= ;; esac
        timeout -k 10 150 python3 tools/power_run.py --label auto -- ./bin/otbench --mode $m --bits $b --bytes 4G $ip \
            --iters 700 --warmup 20 --verify --mark >> $O/energy.jsonl 2>> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
    done
done
python3 - $O/energy.jsonl <<'PY'
import json, sys
print(f'{"mode":12s} {"bits":>4s} {"GB/s":>8s} {"W":>7s} {"J/GB":>6s} {"PPT":>5s} {"MHz":>6s} verified')
for l in open(sys.argv[1]):
    d = json.loads(l); p = d["power"]
    w = p.get("avg_socket_w")
    print(f'{d["mode"]:12s} {d["bits"]:4d} {d["gbps"]:8.1f} {w:7.1f} {w / d["gbps"]:6.3f} {p.get("ppt_residency"):5.2f} '
          f'{p.get("gfxclk_mhz_mean"):6.0f} {d["verified"]}')
PY
