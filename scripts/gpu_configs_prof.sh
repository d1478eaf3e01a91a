# rocprofv3 kernel-trace summaries of bench_configs.py per configuration (CONFIGS, default c1 c2 c3 c5).
set -o pipefail
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in ${CONFIGS:-c1 c2 c3 c5}; do
  mkdir -p $R/gpurun_out/cfg_$c
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/cfg_$c -o run -- python3 $R/bench_configs.py $c > $R/gpurun_out/cfg_$c/bench.log 2>&1 || { echo FAIL $c; tail -5 $R/gpurun_out/cfg_$c/bench.log; exit 1; }
  tail -1 $R/gpurun_out/cfg_$c/bench.log
done
