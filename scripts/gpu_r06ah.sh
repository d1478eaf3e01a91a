# Round 6: C5 -- the batch readback carries the table occupancy (no counter read-back sync on pipelined sizing),
# no sweep event, slot pass before the previous readback (product) vs the r06 host flow; session tests; host
# profile and kernel trace of the product.
set -o pipefail
cd $GRAFT_REPO_ROOT
LIBS="product env:GWO_SESS_FIRE_EVENT=1,GWO_SESS_WM_RESOLVE=1,GWO_SESS_EARLY_SLOT=0" CFG=c5 REPS=3 bash scripts/gpu_cfg_ab.sh || exit 1
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q -k "sess or c5 or merging or multi_round or java or heap_state or checkpoint or pipelined" --timeout 200 --timeout-method thread > gpurun_out/cfgab/pytest_ah.log 2>&1
echo "tests rc=$?"; tail -n 3 gpurun_out/cfgab/pytest_ah.log
mkdir -p gpurun_out/r06ah
GWO_SESS_HOST_PROF=1 BENCH_PROF=0 BENCH_HOST_TIMING=1 timeout -k 10 200 python3 -u bench_configs.py c5 > gpurun_out/r06ah/host.log 2>&1 || exit 1
grep -E 'host us|session host' gpurun_out/r06ah/host.log
cd /tmp && export TMPDIR=/tmp
BENCH_PROF=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06ah/trace -o run -- python3 $GRAFT_REPO_ROOT/bench_configs.py c5 > $GRAFT_REPO_ROOT/gpurun_out/r06ah/trace.log 2>&1
echo "trace rc=$?"
