# Round 6: C5 -- no event behind the watermark sweep (product; its readback word is the completion test) vs the
# event (GWO_SESS_FIRE_EVENT=1) vs the r06 host flow (event, watermark reads the readback, slot pass after it);
# session tests; a kernel trace of the product.
set -o pipefail
cd $GRAFT_REPO_ROOT
LIBS="product env:GWO_SESS_FIRE_EVENT=1 env:GWO_SESS_FIRE_EVENT=1,GWO_SESS_WM_RESOLVE=1,GWO_SESS_EARLY_SLOT=0" CFG=c5 REPS=3 bash scripts/gpu_cfg_ab.sh || exit 1
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q -k "sess or c5 or merging or multi_round or java or heap_state or checkpoint or pipelined" --timeout 200 --timeout-method thread > gpurun_out/cfgab/pytest_af.log 2>&1
echo "tests rc=$?"; tail -n 3 gpurun_out/cfgab/pytest_af.log
cd /tmp && export TMPDIR=/tmp
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/r06af
BENCH_PROF=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06af/trace -o run -- python3 $GRAFT_REPO_ROOT/bench_configs.py c5 > $GRAFT_REPO_ROOT/gpurun_out/r06af/trace.log 2>&1
echo "trace rc=$?"
