# rocprofv3 kernel + HIP runtime API trace of bench_configs.py per configuration (CONFIGS), no PMC counters.
set -o pipefail
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
for c in ${CONFIGS:-c1 c2}; do
  mkdir -p $R/gpurun_out/trace_$c
  BENCH_PROF=0 timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/trace_$c -o run -- python3 $R/bench_configs.py $c > $R/gpurun_out/trace_$c.log 2>&1 || { echo TRACE_FAIL $c; tail -30 $R/gpurun_out/trace_$c.log; exit 1; }
  grep '^{' $R/gpurun_out/trace_$c.log | tail -1
done
