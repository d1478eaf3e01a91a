# Round 6: the bounce-buffer copies (tests/test_gpu_xfer.py), then the whole GPU suite once.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_xfer.py tests/test_gpu_log_lateness.py -m gpu -v -x --timeout 200 --timeout-method thread \
    > $O/pytest_xfer.log 2>&1
rc=$?
tail -12 $O/pytest_xfer.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --durations=15 --timeout 200 --timeout-method thread \
    > $O/pytest_all.log 2>&1
rc=$?
tail -25 $O/pytest_all.log
exit $rc
