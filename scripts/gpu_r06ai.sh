# Round 6: host profiles (GWO_HOST_PROF points, per-call times) of C2 and C1, and C5 again.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06ai
for c in c2 c1 c5; do
  GWO_HOST_PROF=1 BENCH_PROF=0 BENCH_HOST_TIMING=1 timeout -k 10 200 python3 -u bench_configs.py $c > gpurun_out/r06ai/$c.log 2>&1 || exit 1
  echo "[$c]"; grep -E 'host us' gpurun_out/r06ai/$c.log; tail -n 1 gpurun_out/r06ai/$c.log | cut -c1-330 | grep -o '"ms_per_step": [0-9.]*'
done
