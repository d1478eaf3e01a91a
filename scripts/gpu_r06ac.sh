# Round 6: C5 -- the process kernel instantiated per plan word count (product) vs run-time word loops (exp/nwrt),
# 3 rounds; then the session tests on the product.
set -o pipefail
cd $GRAFT_REPO_ROOT
LIBS="exp/nwrt/libgwo.so product" CFG=c5 REPS=3 bash scripts/gpu_cfg_ab.sh || exit 1
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -k "sess or c5 or merging or multi_round or java or heap_state or checkpoint" --timeout 200 --timeout-method thread > gpurun_out/cfgab/pytest_nwt.log 2>&1
echo "product tests rc=$?"; tail -n 1 gpurun_out/cfgab/pytest_nwt.log
