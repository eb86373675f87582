#!/bin/bash
# Final validation of the round's build on one MI355X: smoke(), the whole GPU
# test suite, the bench line, the J/GB power probe, the verified mode sweep and
# the energy table.   gpurun --timeout 1200 -- bash scripts/r4_final.sh NAME
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
N=${1:-r4_final}
O=gpurun_out/$N
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 ||
    { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash scripts/r4_validate.sh $N/validate && bash scripts/sweep.sh $N/sweep && bash scripts/r4_energy_table.sh $N/energy
