# One gpurun call: the GPU tests named in $TESTS (default: all), each under the per-test limit; a crash or
# timeout (rc >= 124) ends the script.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest ${TESTS:-tests} -m gpu -v -x${KEXPR:+ -k "$KEXPR"} --durations=15 \
    --timeout ${PER_TEST:-180} --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_gpu.log
exit $rc
