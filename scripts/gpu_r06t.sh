# Round 6: C2 merge run length A/B (exp/mr4, exp/mr2: CB_MERGE_RUN 4, 2; product 8), 2 rounds; then the combine-path
# tests on both variants.
set -o pipefail
cd $GRAFT_REPO_ROOT
LIBS="product exp/mr4/libgwo.so exp/mr2/libgwo.so" CFG=c2 REPS=2 bash scripts/gpu_cfg_ab.sh || exit 1
for L in exp/mr4/libgwo.so exp/mr2/libgwo.so; do
  GWO_LIB_PATH=$L timeout -k 10 300 python3 -u -m pytest tests/test_gpu_windows.py tests/test_gpu_fullscale_configs.py -m gpu -x -q -k "combine or c2 or table" --timeout 200 --timeout-method thread > gpurun_out/cfgab/pytest_$(basename $(dirname $L)).log 2>&1
  echo "$L tests rc=$?"; tail -n 1 gpurun_out/cfgab/pytest_$(basename $(dirname $L)).log
done
