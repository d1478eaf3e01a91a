# One gpurun call: every GPU test (no -x: all failures are reported), then smoke and a bench line, each step under
# its own limit; a crash/timeout (rc >= 124) stops the script.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest ${TESTS:-tests} -m gpu -v --durations=25 --timeout ${PER_TEST:-240} --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ge 124 ]; then echo "PYTEST rc=$rc: stopping"; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
exit $rc
