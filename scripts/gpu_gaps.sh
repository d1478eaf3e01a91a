# Kernel + copy + HIP API trace of a short bench run, then the per-step GPU gap summary (scripts/gaps.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/trace; mkdir -p $R/gpurun_out/trace
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $R/gpurun_out/trace -o run -- python3 $R/bench.py --steps 10 --warmup 12 --no-cpu-baseline ${BENCH_ARGS:-} > $R/gpurun_out/trace_bench.log 2>&1 || { echo TRACE_FAIL; tail -30 $R/gpurun_out/trace_bench.log; exit 1; }
tail -1 $R/gpurun_out/trace_bench.log | cut -c1-300
