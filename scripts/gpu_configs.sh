# Throughput of configs c1/c2/c3/c5 (bench_configs.py), one process per config, each under its own limit.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/configs.jsonl
for c in ${CONFIGS:-c1 c2 c3 c5}; do
  timeout -k 10 ${LIMIT:-240} python -u bench_configs.py $c > gpurun_out/config_$c.log 2>&1 || { echo FAIL $c; tail -8 gpurun_out/config_$c.log; exit 1; }
  tail -1 gpurun_out/config_$c.log >> gpurun_out/configs.jsonl
  tail -1 gpurun_out/config_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'], round(d['value']/1e9,3), 'G rec/s', round(d['ms_per_step'],3), 'ms/step', {k: round(v['total_ms'],2) for k,v in d['kernels_ms'].items()})"
done
