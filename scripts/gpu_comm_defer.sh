# Deferred receives of the routed exchange: GPU parity of the virtual-rank / watermark tests, then the C4 bench at
# 8 and 2 virtual ranks with and without deferral (GWO_COMM_DEFER), then (ALL=1) the whole GPU suite + smoke + bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/comm
cd $R
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_windows.py tests/test_gpu_watermarks.py -k "comm or virtual" > gpurun_out/comm/pytest.log 2>&1 || { tail -40 gpurun_out/comm/pytest.log; exit 1; }
tail -2 gpurun_out/comm/pytest.log
for v in v8d1 v8d0 v2d1 single; do
  case $v in
    v8d1) args="--comm-single --comm-virtual 8"; d=1;;
    v8d0) args="--comm-single --comm-virtual 8"; d=0;;
    v2d1) args="--comm-single --comm-virtual 2"; d=1;;
    single) args="--comm-single"; d=1;;
  esac
  GWO_COMM_DEFER=$d timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-fed $args > gpurun_out/comm/bench_$v.log 2>&1 || { echo FAIL $v; tail -20 gpurun_out/comm/bench_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/comm/bench_$v.log').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e9,2), 'G rec/s', round(d['ms_per_step'],4), 'ms/step', d.get('kernels_ms'))"
done
if [ "${CFG:-0}" = 1 ]; then bash scripts/gpu_configs.sh || exit 1; fi
if [ "${ALL:-0}" = 1 ]; then TEST_TIMEOUT=700 bash scripts/gpu_all.sh; fi
