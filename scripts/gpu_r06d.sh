# Round 6: the fire's direct-result emit (FireArgs.direct) -- log-layout parity tests, then the C4 A/B against
# GWO_FIRE_DIRECT=0 (the plan-dispatch emit).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullscale.py tests/test_gpu_windows.py tests/test_gpu_log_lateness.py tests/test_gpu_checkpoint.py \
    -m gpu -v -x -k "c4_full_window or log or sharded" --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -6 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
ENVS="base GWO_FIRE_DIRECT=0" REPS=2 bash scripts/gpu_env_ab.sh
