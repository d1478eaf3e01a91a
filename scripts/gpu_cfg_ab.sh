# A/B of library variants on bench_configs.py configurations: CONFIGS (default c2), VARIANTS (base = flink_amd/libgwo.so).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/cfgab
for c in ${CONFIGS:-c2}; do
  for v in ${VARIANTS:-base}; do
    if [ "$v" = base ]; then L=""; else L=$R/exp/$v/libgwo.so; fi
    GWO_LIB_PATH=$L timeout -k 10 300 python3 -u bench_configs.py $c > gpurun_out/cfgab/${c}_$v.log 2>&1 || { echo "FAIL $c $v"; tail -20 gpurun_out/cfgab/${c}_$v.log; exit 1; }
    tail -n 1 gpurun_out/cfgab/${c}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c $v', 'G rec/s %.2f' % (d['value']/1e9), 'ms/step %.4f' % d['ms_per_step'], {k: round(x['total_ms']/max(x['launches'],1)*1e3,1) for k,x in d['kernels_ms'].items()})"
  done
done
