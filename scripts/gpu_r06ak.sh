# Round 6: readback spins query the stream after 500 us (product) instead of every ~30 us (GWO_SPIN_QUERY_US=30,
# the old cadence) -- C2, C1, C5, C4; then a C2 trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
LIBS="product env:GWO_SPIN_QUERY_US=30" CFG=c2 REPS=3 bash scripts/gpu_cfg_ab.sh || exit 1
LIBS="product env:GWO_SPIN_QUERY_US=30" CFG=c1 REPS=2 bash scripts/gpu_cfg_ab.sh || exit 1
LIBS="product env:GWO_SPIN_QUERY_US=30" CFG=c5 REPS=2 bash scripts/gpu_cfg_ab.sh || exit 1
for v in "" "GWO_SPIN_QUERY_US=30"; do
  env $v timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/cfgab/c4_$v.log 2>&1 || exit 1
  echo "C4 [$v] $(tail -n 1 gpurun_out/cfgab/c4_$v.log | grep -o '"ms_per_step": [0-9.]*')"
done
cd /tmp && export TMPDIR=/tmp
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/r06ak
BENCH_PROF=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06ak/trace -o run -- python3 $GRAFT_REPO_ROOT/bench_configs.py c2 > $GRAFT_REPO_ROOT/gpurun_out/r06ak/trace.log 2>&1
echo "trace rc=$?"
