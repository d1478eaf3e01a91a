# 8 virtual ranks: the fire on the handle's stream vs on its own stream (GWO_ASYNC_FIRE=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/async
for af in 0 1; do
  GWO_ASYNC_FIRE=$af timeout -k 10 150 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host-fed --comm-single --comm-virtual 8 > gpurun_out/async/v8_af$af.log 2>&1 || { echo FAIL; tail -20 gpurun_out/async/v8_af$af.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/async/v8_af$af.log').read().strip().splitlines()[-1]); print('v8 async_fire=$af', round(d['value']/1e9,2), 'G rec/s', round(d['ms_per_step'],4), 'ms/step')"
done
