# Selected GPU tests (PYTEST_K) with per-test timeouts.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -k "${PYTEST_K}" > gpurun_out/pytest_k.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_k.log; exit 1; }
tail -12 gpurun_out/pytest_k.log
