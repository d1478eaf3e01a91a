# Round 6: the direct emit's unconditional value reads per row (exp/ev6, exp/ev8: FIRE_EMIT_V 6, 8; product 4) on
# C4, 2 rounds, then the log-layout parity tests on both variants.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06r
mkdir -p $O
for rep in 1 2; do
  for L in product exp/ev6/libgwo.so exp/ev8/libgwo.so; do
    tag=$(echo $L | tr '/' '_'); lp=$L; [ $L = product ] && lp=
    GWO_LIB_PATH=$lp timeout -k 10 240 python3 -u bench.py --steps 20 --warmup 3 --no-host-fed --no-cpu-baseline > $O/$tag.$rep.log 2>&1 || { echo FAIL $L; tail -20 $O/$tag.$rep.log; exit 1; }
    tail -n 1 $O/$tag.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L', 'ms/step %.4f' % d['ms_per_step'], 'K1 %.1f us' % (d['roofline']['avg_launch_ms']*1e3), {k: round(v['total_ms']/max(v['launches'],1),4) for k,v in d['kernels_ms'].items()})"
  done
done
for L in exp/ev6/libgwo.so exp/ev8/libgwo.so; do
  GWO_LIB_PATH=$L timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fullscale.py tests/test_gpu_windows.py tests/test_gpu_sliding_log.py -m gpu -x -q -k "log or c4 or sharded" --timeout 200 --timeout-method thread > $O/pytest_$(basename $(dirname $L)).log 2>&1
  echo "$L tests rc=$?"; tail -n 2 $O/pytest_$(basename $(dirname $L)).log
done
