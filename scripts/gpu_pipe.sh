# Pipelined combine submission: its GPU tests, then C1/C2 with and without pipelining (BENCH_PIPE), then (ALL=1) the
# whole GPU suite + smoke + bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pipe
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu tests/test_gpu_windows.py tests/test_gpu_fullscale_configs.py -k "pipelined" > gpurun_out/pipe/pytest.log 2>&1 || { tail -40 gpurun_out/pipe/pytest.log; exit 1; }
tail -2 gpurun_out/pipe/pytest.log
for p in 1 0; do
  BENCH_PIPE=$p timeout -k 10 200 python3 -u bench_configs.py c2 c1 > gpurun_out/pipe/cfg_p$p.log 2>&1 || { echo FAIL $p; tail -20 gpurun_out/pipe/cfg_p$p.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/pipe/cfg_p$p.log'):
    if l.startswith('{'):
        d=json.loads(l); print('pipe=$p', d['config']['workload'][:2], round(d['value']/1e9,3), 'G rec/s', round(d['ms_per_step']*1e3,1), 'us/step', d['kernels_ms'])"
done
if [ "${ALL:-0}" = 1 ]; then TEST_TIMEOUT=700 bash scripts/gpu_all.sh; fi
