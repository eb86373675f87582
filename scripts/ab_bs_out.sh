# A/B of bitsliced launch structure knobs; run through gpurun
#   VARIANTS="name:ENV=VAL,ENV2=VAL ..."   MODES="ctr ecb"
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "bitslice or bs" > gpurun_out/ab/pytest.log 2>&1 || { tail -30 gpurun_out/ab/pytest.log; exit 1; }
tail -2 gpurun_out/ab/pytest.log
for rep in 1 2; do for mode in ${MODES:-ctr}; do for v in ${VARIANTS:-default:X=0}; do
  name=${v%%:*}; envs=${v#*:}
  env ${envs//,/ } timeout -k 10 120 ./bin/otbench --mode $mode --impl bitslice --bytes ${BYTES:-4G} --iters 20 --clock --verify \
    | sed "s/^/$name /" | tee -a gpurun_out/ab/ab.txt || exit 1
done; done; done
