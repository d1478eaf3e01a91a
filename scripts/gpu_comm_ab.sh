# Routed-K1 exchange: GPU parity (virtual ranks, 1-rank comm) and C4 bench without a communicator, with a 1-rank
# communicator, and with 2 / 8 virtual ranks (a rank's multi-GPU data path measured on one GPU).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/comm
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_windows.py -k "comm" > gpurun_out/comm/pytest.log 2>&1 || { tail -30 gpurun_out/comm/pytest.log; exit 1; }
tail -2 gpurun_out/comm/pytest.log
for v in none single v2 v8; do
  case $v in
    none) args="";;
    single) args="--comm-single";;
    v2) args="--comm-single --comm-virtual 2";;
    v8) args="--comm-single --comm-virtual 8";;
  esac
  timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-fed $args > gpurun_out/comm/bench_$v.log 2>&1 || { echo FAIL $v; tail -20 gpurun_out/comm/bench_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/comm/bench_$v.log').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e9,2), 'G rec/s', round(d['ms_per_step'],4), 'ms/step', d.get('kernels_ms'))"
done
