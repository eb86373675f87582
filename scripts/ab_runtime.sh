#!/bin/bash
# Interleaved A/B over HIP runtimes x variant libraries x otbench configs, with
# energy (tools/power_run.py), every run verified and carrying otbench's
# "runtime" record (A/Bs across two runtimes).
#   rt72  /opt/rocm's HIP 7.2 + RCCL (what otbench and the CLIs bind by default)
#   rt70  torch's bundled HIP 7.0 + RCCL (what bench.py and pytest bind): the
#         files in torch/lib, linked under their SONAMEs into a directory put
#         first on LD_LIBRARY_PATH, so libotc.so's NEEDED entries resolve there
# Run on the box:
#   bash scripts/ab_runtime.sh OUT REPS "rt70 rt72" "otbench args;..." variant1 variant2 ...
# ("base" = a copy of the default build, made here) -> gpurun_out/OUT/ab.jsonl
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=$1; reps=$2; rts=$3; cfgs=$4; shift 4
O=gpurun_out/$out
mkdir -p $O variants/base
[ -f variants/base/libotc.so ] || cp our_tree_amd/lib/libotc.so variants/base/
TL=/usr/local/lib/python3.10/dist-packages/torch/lib
R70=/tmp/otc_rt70
mkdir -p $R70
for f in libamdhip64.so libhsa-runtime64.so librccl.so libamd_comgr.so librocprofiler-register.so; do
    [ -f $TL/$f ] || continue
    so=$(readelf -d $TL/$f | sed -n 's/.*(SONAME).*\[\(.*\)\]/\1/p')
    [ -n "$so" ] && ln -sf $TL/$f $R70/$so
done
IFS=';' read -ra CFG <<< "$cfgs"
for r in $(seq 1 "$reps"); do for c in "${CFG[@]}"; do for rt in $rts; do for v in "$@"; do
    if [ "$rt" = rt70 ]; then LP=$R70:variants/$v; else LP=variants/$v; fi
    LD_LIBRARY_PATH=$LP timeout -k 10 150 python3 tools/power_run.py --label "$v/$rt" -- \
        ./bin/otbench $c --verify --mark >> $O/ab.jsonl 2>> $O/err.txt || { echo "FAILED $v $rt $c"; tail -5 $O/err.txt; exit 1; }
    python3 - "$O/ab.jsonl" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
p = d["power"]
rt = d.get("runtime") or {}
print(f'{d["label"]:14s} hip {rt.get("hip_runtime_version")} {d["mode"]:8s} {d["bits"]} {d["bytes"] >> 30:3d}G '
      f'{d["impl"]}->{d.get("ran")} {d["gbps"]:8.1f} GB/s v={d["verified"]} {p.get("avg_socket_w")} W '
      f'{d.get("joules_per_gb")} J/GB gfx {p.get("gfxclk_mhz_mean")} MHz' +
      (f' units {d["split_units"]}' if "split_units" in d else ''), flush=True)
PY
done; done; done; done
