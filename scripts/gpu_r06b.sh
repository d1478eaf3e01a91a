# Round 6: the tests changed this round (checkpoint dedup, Java mirror lifetime, watermark flow-control bounds).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_checkpoint.py tests/test_gpu_java_sequence.py tests/test_gpu_watermarks.py \
    -m gpu -v -rA --durations=10 --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|routed [0-9]+:" $O/pytest.log | tail -60
tail -15 $O/pytest.log
exit $rc
