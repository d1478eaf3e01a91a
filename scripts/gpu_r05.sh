# One gpurun call for round 5 checks: the GPU tests named in $TESTS (default: all), then (unless NO_BENCH) the C4
# bench line; each step under its own limit, the call stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/${OUT:-r05}
timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest ${TESTS:-tests} -m gpu -v -x${KEXPR:+ -k "$KEXPR"} --durations=15 \
    --timeout ${PER_TEST:-180} --timeout-method thread > gpurun_out/${OUT:-r05}/pytest_gpu.log 2>&1
rc=$?
tail -25 gpurun_out/${OUT:-r05}/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "PYTEST rc=$rc: stopping"; exit $rc; fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/${OUT:-r05}/bench.json 2> gpurun_out/${OUT:-r05}/bench.err || { echo "bench failed"; tail -20 gpurun_out/${OUT:-r05}/bench.err; exit 1; }
  cat gpurun_out/${OUT:-r05}/bench.json
fi
