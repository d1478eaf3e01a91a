# Round 6: C5 -- the sweep's two statistics words folded in one round of exchanges (product) vs one after the other
# (exp/base = HEAD); session tests on the product.
set -o pipefail
cd $GRAFT_REPO_ROOT
LIBS="product exp/base/libgwo.so" CFG=c5 REPS=4 bash scripts/gpu_cfg_ab.sh || exit 1
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q -k "sess or c5 or merging or multi_round or java or heap_state or checkpoint or pipelined" --timeout 200 --timeout-method thread > gpurun_out/cfgab/pytest_ap.log 2>&1
echo "tests rc=$?"; tail -n 2 gpurun_out/cfgab/pytest_ap.log
