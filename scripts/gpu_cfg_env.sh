# A/B of environment settings on one bench_configs.py configuration (CFG, default c3): ENVS="A=1 A=0,B=2 base".
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/cfgenv
for e in ${ENVS:-base}; do
  tag=$(echo "$e" | tr ',=' '_-')
  env $(echo "$e" | tr ',' ' ' | sed 's/^base$//') GWO_LIB_PATH=${LIB:-} timeout -k 10 240 python3 -u bench_configs.py ${CFG:-c3} > gpurun_out/cfgenv/$tag.log 2>&1 || { echo "FAIL $e"; tail -20 gpurun_out/cfgenv/$tag.log; exit 1; }
  tail -n 1 gpurun_out/cfgenv/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$e', 'G rec/s %.2f' % (d['value']/1e9), 'ms/step %.4f' % d['ms_per_step'], {k: round(x['total_ms']/max(x['launches'],1)*1e3,1) for k,x in d['kernels_ms'].items()})"
done
