# Round 6: the session kernels' readback in one round of atomics (product) vs the fold-then-add tails (exp/sold = the
# previous commit's kernels), C5, 3 rounds; then the session tests on the product.
set -o pipefail
cd $GRAFT_REPO_ROOT
LIBS="exp/sold/libgwo.so product" CFG=c5 REPS=3 bash scripts/gpu_cfg_ab.sh || exit 1
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -k "sess or c5 or merging or multi_round" --timeout 200 --timeout-method thread > gpurun_out/cfgab/pytest_sess.log 2>&1
echo "product tests rc=$?"; tail -n 1 gpurun_out/cfgab/pytest_sess.log
