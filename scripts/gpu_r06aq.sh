# Round 6: C5 -- the long kernel's readback in one round of atomics (product) vs fold-then-returning-add (exp/fold2,
# which has the sweep's two-word fold) vs HEAD (exp/base); session tests on the product.
set -o pipefail
cd $GRAFT_REPO_ROOT
LIBS="product exp/fold2/libgwo.so exp/base/libgwo.so" CFG=c5 REPS=4 bash scripts/gpu_cfg_ab.sh || exit 1
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q -k "sess or c5 or merging or multi_round or java or heap_state or checkpoint or pipelined" --timeout 200 --timeout-method thread > gpurun_out/cfgab/pytest_aq.log 2>&1
echo "tests rc=$?"; tail -n 2 gpurun_out/cfgab/pytest_aq.log
