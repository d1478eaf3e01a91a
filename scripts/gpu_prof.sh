# rocprofv3 kernel-trace summary of a short bench run (copied into profiles/ afterwards).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-12} --no-cpu-baseline > $R/gpurun_out/prof_bench.log 2>&1 || { echo PROF_FAIL; tail -30 $R/gpurun_out/prof_bench.log; exit 1; }
tail -1 $R/gpurun_out/prof_bench.log
find $R/gpurun_out/prof -name "*stats.csv" | head
