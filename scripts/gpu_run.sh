# One gpurun call: GPU tests (TESTS, default all; "none" skips), a bench line (BENCH = bench.py args) and a
# rocprofv3 kernel-trace summary of a bench command (PROF = bench.py args), each step under its own limit.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
if [ "$TESTS" != none ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -m gpu -v -x --timeout ${PER_TEST:-300} --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 1; }
  cat gpurun_out/smoke.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python -u bench.py $BENCH > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench.log; exit 1; }
  tail -1 gpurun_out/bench.log
fi
if [ -n "$PROF" ]; then
  mkdir -p $R/gpurun_out/prof
  export TMPDIR=/tmp
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py $PROF > $R/gpurun_out/prof_bench.log 2>&1 || { echo PROF_FAIL; tail -30 $R/gpurun_out/prof_bench.log; exit 1; }
  tail -1 $R/gpurun_out/prof_bench.log
fi
