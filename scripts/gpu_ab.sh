# A/B of library variants (exp/NAME/libgwo.so via GWO_LIB_PATH; "base" = flink_amd/libgwo.so) on the C4 bench:
# VARIANTS="base trace ..." BENCH_ARGS="..." ; each run under its own limit, traced variants print [ktrace] sums.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/ab
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then L=""; else L=$R/exp/$v/libgwo.so; fi
  GWO_LIB_PATH=$L GWO_KTRACE=1 timeout -k 10 240 python3 -u bench.py ${BENCH_ARGS:---steps 12 --warmup 2 --no-host-fed --no-cpu-baseline} > gpurun_out/ab/$v.log 2>&1 || { echo "FAIL $v"; tail -20 gpurun_out/ab/$v.log; exit 1; }
  echo "== $v"; grep -v '^{' gpurun_out/ab/$v.log | grep -v amdgpu.ids
  tail -n 1 gpurun_out/ab/$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step %.4f' % d['ms_per_step'], {k: round(v['total_ms']/max(v['launches'],1),4) for k,v in d['kernels_ms'].items()})"
done
