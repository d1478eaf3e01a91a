# Cost of the per-kernel profiling events: bench with and without them, twice, same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for f in "" "--no-profile" "" "--no-profile"; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline $f > gpurun_out/ev.log 2>&1 || { echo BENCH_FAIL $f; tail -20 gpurun_out/ev.log; exit 1; }
  tail -1 gpurun_out/ev.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value']/1e9,2), round(d['ms_per_step'],3))"
done
