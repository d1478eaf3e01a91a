# Round 6: C2 -- the gather tail reads the previous batch's verdict in its first round of atomics (product) vs at
# the verdict (exp/base = HEAD); combine tests on the product.
set -o pipefail
cd $GRAFT_REPO_ROOT
LIBS="product exp/base/libgwo.so" CFG=c2 REPS=4 bash scripts/gpu_cfg_ab.sh || exit 1
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q -k "combine or c2 or pipelined or tumbling" --timeout 200 --timeout-method thread > gpurun_out/cfgab/pytest_as.log 2>&1
echo "tests rc=$?"; tail -n 2 gpurun_out/cfgab/pytest_as.log
