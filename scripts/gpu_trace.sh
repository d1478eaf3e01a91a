# rocprofv3 kernel + HIP runtime API trace of a short bench run (no PMC counters in this pass).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/trace
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d $R/gpurun_out/trace -o run -- python3 $R/bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-12} --no-cpu-baseline ${BENCH_ARGS:-} > $R/gpurun_out/trace_bench.log 2>&1 || { echo TRACE_FAIL; tail -30 $R/gpurun_out/trace_bench.log; exit 1; }
tail -1 $R/gpurun_out/trace_bench.log
ls $R/gpurun_out/trace
