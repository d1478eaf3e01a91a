# Round 6: C3 with pipelined submission (BENCH_PIPE=1) vs without; host per-call times of both.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06am
for rep in 1 2; do
  for p in 0 1; do
    BENCH_PIPE=$p BENCH_PROF=0 BENCH_HOST_TIMING=1 timeout -k 10 300 python3 -u bench_configs.py c3 > gpurun_out/r06am/c3_pipe$p.$rep.log 2>&1 || exit 1
    echo "pipe=$p $(tail -n 1 gpurun_out/r06am/c3_pipe$p.$rep.log | grep -o '"ms_per_step": [0-9.]*') $(grep 'host us' gpurun_out/r06am/c3_pipe$p.$rep.log)"
  done
done
