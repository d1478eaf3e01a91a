# Round 6: C5 -- process workgroups of 1 (product) / 2 / 4 waves (exp/pw2, exp/pw4), 3 rounds; session tests on pw4.
set -o pipefail
cd $GRAFT_REPO_ROOT
LIBS="product exp/pw2/libgwo.so exp/pw4/libgwo.so" CFG=c5 REPS=3 bash scripts/gpu_cfg_ab.sh || exit 1
GWO_LIB_PATH=exp/pw4/libgwo.so timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -k "sess or c5 or merging or multi_round" --timeout 200 --timeout-method thread > gpurun_out/cfgab/pytest_pw4.log 2>&1
echo "pw4 tests rc=$?"; tail -n 1 gpurun_out/cfgab/pytest_pw4.log
