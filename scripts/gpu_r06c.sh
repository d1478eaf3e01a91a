# Round 6: pass 2 on its own stream (GWO_SPLIT_STREAM=1) -- the log-layout parity tests under it, then the C4 A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06c
mkdir -p $O
GWO_SPLIT_STREAM=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_fullscale.py tests/test_gpu_log_lateness.py tests/test_gpu_checkpoint.py \
    -m gpu -v -x -k "c4_full_window or sharded or log" --timeout 180 --timeout-method thread > $O/pytest_split.log 2>&1
rc=$?
tail -6 $O/pytest_split.log
[ $rc -eq 0 ] || exit $rc
ENVS="base GWO_SPLIT_STREAM=1" REPS=2 bash scripts/gpu_env_ab.sh
