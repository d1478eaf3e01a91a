# Round 6: the new pipelined-session release / table-growth test and its neighbours.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06ao
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_windows.py -m gpu -x -v -k "pipelined" --timeout 200 --timeout-method thread > gpurun_out/r06ao/pytest.log 2>&1
rc=$?; tail -n 12 gpurun_out/r06ao/pytest.log; exit $rc
