# One gpurun call: GPU tests, the default bench line, then the 8-virtual-rank exchange bench.
# Each GPU step under its own time limit; the call stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -v --durations=25 --timeout ${PER_TEST:-300} --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "PYTEST rc=$rc: stopping"; exit $rc; fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
if [ -n "$COMM" ]; then
  timeout -k 10 300 python -u bench.py --comm-single --comm-virtual 8 --no-cpu-baseline --no-host-fed > gpurun_out/comm_v8.json 2> gpurun_out/comm_v8.err || { echo "comm bench failed"; tail -20 gpurun_out/comm_v8.err; exit 1; }
  cat gpurun_out/comm_v8.json
fi
