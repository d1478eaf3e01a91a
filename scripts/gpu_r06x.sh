# Round 6: LDS-only barriers in the K1, gather and scan tails (product) vs __syncthreads (exp/tailold): C4 3 rounds,
# C2 3 rounds, C1 2 rounds; then the log-layout and combine-path tests on the product.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06x
mkdir -p $O
for rep in 1 2 3; do
  for L in exp/tailold/libgwo.so product; do
    tag=$(echo $L | tr '/' '_'); lp=$L; [ $L = product ] && lp=
    GWO_LIB_PATH=$lp timeout -k 10 240 python3 -u bench.py --steps 20 --warmup 3 --no-host-fed --no-cpu-baseline > $O/$tag.$rep.log 2>&1 || { echo FAIL $L; tail -20 $O/$tag.$rep.log; exit 1; }
    tail -n 1 $O/$tag.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C4 $L', 'ms/step %.4f' % d['ms_per_step'], 'K1 %.1f us' % (d['roofline']['avg_launch_ms']*1e3), {k: round(v['total_ms']/max(v['launches'],1),4) for k,v in d['kernels_ms'].items()})"
  done
done
LIBS="exp/tailold/libgwo.so product" CFG=c2 REPS=3 bash scripts/gpu_cfg_ab.sh || exit 1
LIBS="exp/tailold/libgwo.so product" CFG=c1 REPS=2 bash scripts/gpu_cfg_ab.sh || exit 1
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_fullscale.py tests/test_gpu_windows.py tests/test_gpu_sliding_log.py tests/test_gpu_checkpoint.py tests/test_gpu_fullscale_configs.py -m gpu -x -q -k "log or c4 or sharded or combine or c2 or table" --timeout 200 --timeout-method thread > $O/pytest_product.log 2>&1
echo "product tests rc=$?"; tail -n 2 $O/pytest_product.log
