# GPU tests selected by -k "$KEXPR" (one pytest process, per-test limit).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 ${LIMIT:-500} python3 -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu tests -k "$KEXPR" > gpurun_out/pytest_k.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_k.log
exit $rc
