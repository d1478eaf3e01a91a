# Round 6, first call: the device-input readiness tests and the sharded union on the product library, then the
# sliding-log tests on the bounds-checked diagnostic builds (exp/chkbig: GWO_SLOG_CHECK + the r05 2048-slot window
# step; exp/chk: GWO_SLOG_CHECK on the product geometry).  A violation is printed as "[slog-check] ..." and skipped.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests/test_gpu_boundary.py tests/test_gpu_fullscale.py tests/test_gpu_sliding_log.py \
    -m gpu -v -x -k "boundary or sharded or sliding_log" --durations=10 --timeout 180 --timeout-method thread \
    > $O/pytest_product.log 2>&1
rc=$?
tail -25 $O/pytest_product.log
[ $rc -eq 0 ] || exit $rc
for v in chkbig chk; do
  GWO_LIB_PATH=$PWD/exp/$v/libgwo.so timeout -k 10 300 python -u -m pytest tests/test_gpu_sliding_log.py \
      tests/test_gpu_fullscale_configs.py -m gpu -v -x -k "sliding_log or c3_sliding_10m_keys_full_scale" \
      --timeout 180 --timeout-method thread > $O/pytest_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"; grep -c "slog-check" $O/pytest_$v.log; grep "slog-check" $O/pytest_$v.log | head -5
  tail -4 $O/pytest_$v.log
  [ $rc -eq 0 ] || exit $rc
done
