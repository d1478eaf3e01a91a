# Round-end measurement set (one gpurun call): the driver's bench command with a rocprofv3 kernel-trace summary,
# PMC traffic passes (FETCH_SIZE, WRITE_SIZE: separate runs), and bench_configs.py per configuration (values
# without per-kernel events, then a rocprofv3 summary).  Every step under its own limit; stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/round
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/round/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/round/bench.log; exit 1; }
tail -1 gpurun_out/round/bench.log
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/round/prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $R/gpurun_out/round/prof_bench.log 2>&1 ) || { echo PROF_FAIL; tail -20 gpurun_out/round/prof_bench.log; exit 1; }
PASSES="FETCH_SIZE;WRITE_SIZE" KREGEX="log_|gather|merge|fire|route" bash scripts/gpu_pmc.sh || exit 1
for c in ${CONFIGS:-c1 c2 c3 c5}; do
  BENCH_PROF=0 timeout -k 10 300 python3 bench_configs.py $c > gpurun_out/round/cfg_$c.log 2>&1 || { echo CFG_FAIL $c; tail -10 gpurun_out/round/cfg_$c.log; exit 1; }
  tail -1 gpurun_out/round/cfg_$c.log
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/round/cfg_$c -o run -- python3 $R/bench_configs.py $c > $R/gpurun_out/round/cfg_${c}_prof.log 2>&1 ) || { echo CFGPROF_FAIL $c; exit 1; }
done
