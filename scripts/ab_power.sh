#!/bin/bash
# Interleaved A/B of variant libraries (make variant NAME=...; variants/NAME/
# libotc.so, "base" = a copy of the default build) with energy: every run goes
# through tools/power_run.py (socket energy, power, PPT residency over the
# timed loop) and is verified.  Run on the box:
#   bash scripts/ab_power.sh OUT REPS "otbench args;otbench args;..." name1 name2 ...
# -> gpurun_out/OUT/ab.jsonl (otbench JSON + variant + power + joules_per_gb)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=$1; reps=$2; cfgs=$3; shift 3
O=gpurun_out/$out
mkdir -p $O
IFS=';' read -ra CFG <<< "$cfgs"
for r in $(seq 1 "$reps"); do for c in "${CFG[@]}"; do for v in "$@"; do
    LD_LIBRARY_PATH=variants/$v timeout -k 10 150 python3 tools/power_run.py --label "$v" -- \
        ./bin/otbench $c --verify --mark >> $O/ab.jsonl 2>> $O/err.txt || { echo "FAILED $v $c"; tail -5 $O/err.txt; exit 1; }
    python3 - "$O/ab.jsonl" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
p = d["power"]
print(f'{d["label"]:8s} {d["mode"]:8s} {d["bits"]} {d["bytes"] >> 30:3d}G {d["gbps"]:8.1f} GB/s v={d["verified"]} '
      f'{p.get("avg_socket_w")} W {d.get("joules_per_gb")} J/GB PPT {p.get("ppt_residency")} '
      f'gfx {p.get("gfxclk_mhz_mean")} MHz' + (f' units {d["split_units"]}' if "split_units" in d else ''), flush=True)
PY
done; done; done
