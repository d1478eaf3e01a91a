# Kernel trace of bench_configs c3 (no per-kernel events): where the step's idle time sits.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c3trace
export TMPDIR=/tmp
cd /tmp
BENCH_PROF=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/c3trace -o run -- python3 $R/bench_configs.py c3 > $R/gpurun_out/c3trace/bench.log 2>&1 || { echo TRACE_FAIL; tail -30 $R/gpurun_out/c3trace/bench.log; exit 1; }
grep '^{' $R/gpurun_out/c3trace/bench.log | cut -c1-200
