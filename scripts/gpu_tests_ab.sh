# One gpurun call: the GPU test suite (all failures reported), then the A/B variants of scripts/gpu_ab.sh.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -v --durations=25 --timeout ${PER_TEST:-300} --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ge 124 ]; then echo "PYTEST rc=$rc: stopping"; exit $rc; fi
bash scripts/gpu_ab.sh || exit 1
exit $rc
