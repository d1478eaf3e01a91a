# Round 6: C2 / C1 -- gwo_kernels.hip built with the basic SGPR allocator (product: no private segment in the
# gather) vs the greedy one (exp/c2old); combine + scan tests on the product; kernel trace of C2.
set -o pipefail
cd $GRAFT_REPO_ROOT
LIBS="product exp/c2old/libgwo.so" CFG=c2 REPS=3 bash scripts/gpu_cfg_ab.sh || exit 1
LIBS="product exp/c2old/libgwo.so" CFG=c1 REPS=2 bash scripts/gpu_cfg_ab.sh || exit 1
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q -k "combine or c2 or c1 or speculative or tumbling or pipelined" --timeout 200 --timeout-method thread > gpurun_out/cfgab/pytest_aj.log 2>&1
echo "tests rc=$?"; tail -n 3 gpurun_out/cfgab/pytest_aj.log
cd /tmp && export TMPDIR=/tmp
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/r06aj
BENCH_PROF=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06aj/trace -o run -- python3 $GRAFT_REPO_ROOT/bench_configs.py c2 > $GRAFT_REPO_ROOT/gpurun_out/r06aj/trace.log 2>&1
echo "trace rc=$?"
