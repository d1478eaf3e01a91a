# Session-path change: its GPU tests, then C5 (A/B: SESS_AB="auto 0 auto 0" runs C5 with GWO_SESS_LISTS per entry).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sess
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu tests -k "session or sess or c5 or merging or pipelined or heap or snapshot or checkpoint" > gpurun_out/sess/pytest.log 2>&1 || { tail -40 gpurun_out/sess/pytest.log; exit 1; }
tail -2 gpurun_out/sess/pytest.log
for m in ${SESS_AB:-auto}; do
  if [ "$m" = auto ]; then unset GWO_SESS_LISTS; else export GWO_SESS_LISTS=$m; fi
  timeout -k 10 200 python3 -u bench_configs.py c5 > gpurun_out/sess/c5_$m.log 2>&1 || { tail -20 gpurun_out/sess/c5_$m.log; exit 1; }
  grep '^{' gpurun_out/sess/c5_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5 lists=$m', round(d['value']/1e9,3), 'G rec/s', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(x['total_ms']/max(x['launches'],1)*1e3,1) for k,x in d['kernels_ms'].items()})"
done
unset GWO_SESS_LISTS
