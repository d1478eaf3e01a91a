# Round 6: fire emit/P3 A/B on C4, 2 rounds: exp/p3old = the previous product (P3 followers read a scattered word,
# FIRE_EMIT_V 4); exp/ev2, exp/ev3 = the same with FIRE_EMIT_V 2, 3; product = P3 followers read word 0
# (FIRE_P3_BCAST); then the log-layout parity tests on the product.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s
mkdir -p $O
for rep in 1 2; do
  for L in exp/p3old/libgwo.so product exp/ev2/libgwo.so exp/ev3/libgwo.so; do
    tag=$(echo $L | tr '/' '_'); lp=$L; [ $L = product ] && lp=
    GWO_LIB_PATH=$lp timeout -k 10 240 python3 -u bench.py --steps 20 --warmup 3 --no-host-fed --no-cpu-baseline > $O/$tag.$rep.log 2>&1 || { echo FAIL $L; tail -20 $O/$tag.$rep.log; exit 1; }
    tail -n 1 $O/$tag.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L', 'ms/step %.4f' % d['ms_per_step'], 'K1 %.1f us' % (d['roofline']['avg_launch_ms']*1e3), {k: round(v['total_ms']/max(v['launches'],1),4) for k,v in d['kernels_ms'].items()})"
  done
done
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fullscale.py tests/test_gpu_windows.py tests/test_gpu_sliding_log.py tests/test_gpu_checkpoint.py -m gpu -x -q -k "log or c4 or sharded" --timeout 200 --timeout-method thread > $O/pytest_product.log 2>&1
echo "product tests rc=$?"; tail -n 2 $O/pytest_product.log
