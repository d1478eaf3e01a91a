# Pipelined-submission check: the new GPU tests, then the bench with and without pipelining.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_pipe.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_pipe.log; exit 1; }
tail -3 gpurun_out/pytest_pipe.log
for f in "" "--pipeline" ""; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline $f > gpurun_out/pipe.log 2>&1 || { echo BENCH_FAIL $f; tail -20 gpurun_out/pipe.log; exit 1; }
  tail -1 gpurun_out/pipe.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value']/1e9,2), round(d['ms_per_step'],3), round(d['roofline_path']['frac'],3), {k: round(v['total_ms']/v['launches'],3) for k,v in d['kernels_ms'].items()})"
done
