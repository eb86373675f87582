#!/bin/bash
# One parametrised GPU runner (run it on the box through gpurun):
#
#   gpurun --timeout 900 -- bash scripts/run.sh <suite> [args...]
#
# suites
#   validate            pytest -m gpu, smoke(), default bench.py   (round-end checks)
#   test [pytest args]  pytest -m gpu (optionally a subset: test tests/test_gpu_engine.py -k cbc)
#   bench [bench args]  bench.py with the given flags
#   rehearse N [args]   bench.py --gpus N --gib 2 self-spawned, N ranks sharing the box's GPU (gloo)
#   kt NAME -- CMD...   rocprofv3 kernel trace + stats of CMD, summarised to gpurun_out/NAME/kernels.txt
#   pmc NAME "COUNTERS" -- CMD...   one counter pass (<= 8 SQ, 4 TCC, ...) of CMD, CSV in gpurun_out/NAME
#   otbench [otbench args]          bin/otbench JSON lines
#   ab "name:ENV=V,ENV2=V name2:..." [otbench args]
#                       A/B: the otbench run once per variant (env knobs), 2 reps
#                       interleaved, lines prefixed with the variant name
#   cmd -- CMD...       anything else, under a time limit
#
# Every GPU step runs under its own `timeout -k 10`, steps are chained with &&
# and the script stops at the first failure (no retries).  Output goes under
# gpurun_out/ (merged back by gpurun); copy what is worth keeping to profiles/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
suite=${1:-validate}
shift || true
OUT=gpurun_out
mkdir -p $OUT

pytest_gpu() {
    timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread "$@"
}

case "$suite" in
validate)
    D=$OUT/validate
    mkdir -p $D
    pytest_gpu tests > $D/pytest_gpu.log 2>&1 || { tail -40 $D/pytest_gpu.log; exit 1; }
    tail -1 $D/pytest_gpu.log
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { cat $D/smoke.log; exit 1; }
    tail -1 $D/smoke.log
    timeout -k 10 600 python bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
    cat $D/bench.json
    ;;
test)
    [ $# -gt 0 ] || set -- tests
    pytest_gpu "$@" > $OUT/pytest_gpu.log 2>&1
    rc=$?
    tail -30 $OUT/pytest_gpu.log
    exit $rc
    ;;
bench)
    timeout -k 10 900 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
    cat $OUT/bench.json
    ;;
rehearse)
    n=${1:-2}
    shift || true
    # N shards must fit ONE GPU: 2 GiB each unless the args say otherwise (argparse keeps the last --gib)
    OTC_DIST_BACKEND=gloo OTC_SHARE_GPUS=1 timeout -k 10 600 python bench.py --gpus "$n" --no-clock --gib 2 "$@" \
        > $OUT/rehearse_dp$n.txt 2>&1 || { tail -30 $OUT/rehearse_dp$n.txt; exit 1; }
    grep '^{' $OUT/rehearse_dp$n.txt | tail -1 > $OUT/rehearse_dp$n.json
    cat $OUT/rehearse_dp$n.json
    # the per-rank table (ranks share one GPU here: their energy keys all read that GPU)
    python3 - $OUT/rehearse_dp$n.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
print(f"{'rank':>4} {'GB/s':>9} {'verified':>8} {'W':>7} {'J/GB':>7} {'PPT':>6}")
for r in d.get("per_rank", []):
    print(f"{r['rank']:>4} {r['gbps']:>9} {str(r['verified']):>8} {str(r['avg_socket_w']):>7} "
          f"{str(r['joules_per_gb']):>7} {str(r['ppt_residency']):>6}")
print("preflight", d.get("preflight"), "rccl_ranks_verified", d.get("rccl_ranks_verified"))
PY
    ;;
kt)
    name=$1; shift; [ "$1" = "--" ] && shift
    mkdir -p $OUT/$name
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/$name/db -o run -- "$@" > $OUT/$name/run.log 2>&1 ||
        { tail -20 $OUT/$name/run.log; exit 1; }
    db=$(find $OUT/$name/db -name '*.db' | head -1)
    python tools/rocpd_summary.py "$db" > $OUT/$name/kernels.txt && cat $OUT/$name/kernels.txt
    ;;
pmc)
    name=$1; counters=$2; shift 2; [ "$1" = "--" ] && shift
    mkdir -p $OUT/$name
    timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d $OUT/$name -o run -- "$@" \
        > $OUT/$name/run.log 2>&1 || { tail -20 $OUT/$name/run.log; exit 1; }
    find $OUT/$name -name '*counter_collection.csv' | head -3
    ;;
otbench)
    timeout -k 10 600 ./bin/otbench "$@" > $OUT/otbench.jsonl 2> $OUT/otbench.err || { tail -20 $OUT/otbench.err; exit 1; }
    cat $OUT/otbench.jsonl
    ;;
ab)
    variants=$1; shift
    for rep in 1 2; do for v in $variants; do
        name=${v%%:*}; envs=${v#*:}
        env ${envs//,/ } timeout -k 10 300 ./bin/otbench "$@" | sed "s/^/$name /" | tee -a $OUT/ab.txt || exit 1
    done; done
    ;;
cmd)
    [ "$1" = "--" ] && shift
    timeout -k 10 900 "$@"
    ;;
*)
    echo "unknown suite: $suite" >&2
    exit 2
    ;;
esac
