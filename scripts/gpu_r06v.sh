# Round 6: the chained verdict loaded at the gather's start (product, CB_EARLY_CHAIN) vs in its tail (exp/chold),
# C2, 3 rounds; then the combine-path tests on the product.
set -o pipefail
cd $GRAFT_REPO_ROOT
LIBS="exp/chold/libgwo.so product" CFG=c2 REPS=3 bash scripts/gpu_cfg_ab.sh || exit 1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_windows.py tests/test_gpu_fullscale_configs.py tests/test_gpu_checkpoint.py -m gpu -x -q -k "combine or c2 or table" --timeout 200 --timeout-method thread > gpurun_out/cfgab/pytest_chain.log 2>&1
echo "product tests rc=$?"; tail -n 1 gpurun_out/cfgab/pytest_chain.log
