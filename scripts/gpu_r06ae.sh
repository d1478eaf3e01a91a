# Round 6: C5 -- the pipelined batch's readback read by the next submit after its slot pass is queued, the watermark
# waiting only for the input-release word (product) vs the watermark reading the readback (old) and vs release-only;
# then the session tests and a kernel trace of the product.
set -o pipefail
cd $GRAFT_REPO_ROOT
LIBS="product env:GWO_SESS_WM_RESOLVE=1,GWO_SESS_EARLY_SLOT=0 env:GWO_SESS_EARLY_SLOT=0" CFG=c5 REPS=3 bash scripts/gpu_cfg_ab.sh || exit 1
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q -k "sess or c5 or merging or multi_round or java or heap_state or checkpoint or pipelined" --timeout 200 --timeout-method thread > gpurun_out/cfgab/pytest_ae.log 2>&1
echo "tests rc=$?"; tail -n 3 gpurun_out/cfgab/pytest_ae.log
for c in c5 c2; do
  BENCH_PROF=0 BENCH_HOST_TIMING=1 timeout -k 10 200 python3 -u bench_configs.py $c > gpurun_out/cfgab/host_$c.log 2>&1 || exit 1
  echo "$c product: $(grep 'host us' gpurun_out/cfgab/host_$c.log)"
done
GWO_SESS_WM_RESOLVE=1 GWO_SESS_EARLY_SLOT=0 BENCH_PROF=0 BENCH_HOST_TIMING=1 timeout -k 10 200 python3 -u bench_configs.py c5 > gpurun_out/cfgab/host_c5_old.log 2>&1 || exit 1
echo "c5 old: $(grep 'host us' gpurun_out/cfgab/host_c5_old.log)"
cd /tmp && export TMPDIR=/tmp
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/r06ae
BENCH_PROF=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r06ae/trace -o run -- python3 $GRAFT_REPO_ROOT/bench_configs.py c5 > $GRAFT_REPO_ROOT/gpurun_out/r06ae/trace.log 2>&1
echo "trace rc=$?"
