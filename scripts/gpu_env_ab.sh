# A/B of environment settings on the C4 bench within one GPU call: ENVS="A=1 A=0 ..." (each entry one run; use
# commas to set several variables in one entry: "A=1,B=2"), REPS rounds; each run under its own limit.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/envab
for rep in $(seq 1 ${REPS:-2}); do
  for e in ${ENVS:-base}; do
    tag=$(echo "$e" | tr ',=' '_-')
    env $(echo "$e" | tr ',' ' ' | sed 's/^base$//') GWO_LIB_PATH=${LIB:-} timeout -k 10 240 python3 -u bench.py ${BENCH_ARGS:---steps 20 --warmup 3 --no-host-fed --no-cpu-baseline} > gpurun_out/envab/$tag.$rep.log 2>&1 || { echo "FAIL $e"; tail -20 gpurun_out/envab/$tag.$rep.log; exit 1; }
    echo "== $e (rep $rep)"; grep -v '^{' gpurun_out/envab/$tag.$rep.log | grep -v amdgpu.ids | tail -12
    tail -n 1 gpurun_out/envab/$tag.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step %.4f' % d['ms_per_step'], 'K1 %.1f us' % (d['roofline']['avg_launch_ms']*1e3), {k: round(v['total_ms']/max(v['launches'],1),4) for k,v in d['kernels_ms'].items()})"
  done
done
