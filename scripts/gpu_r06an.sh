# Round 6: C1 with pipelined submission (BENCH_PIPE=1) vs without (the default), after the spin-query change.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06an
for rep in 1 2 3; do
  for p in 0 1; do
    BENCH_PIPE=$p BENCH_PROF=0 BENCH_HOST_TIMING=1 timeout -k 10 200 python3 -u bench_configs.py c1 > gpurun_out/r06an/c1_pipe$p.$rep.log 2>&1 || exit 1
    echo "pipe=$p $(tail -n 1 gpurun_out/r06an/c1_pipe$p.$rep.log | grep -o '"ms_per_step": [0-9.]*') $(grep 'host us' gpurun_out/r06an/c1_pipe$p.$rep.log | cut -c1-90)"
  done
done
