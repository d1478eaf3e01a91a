# A/B timing of alternative builds of libgwo.so (exp/libgwo_*.so) on the bench workload.
cd $GRAFT_REPO_ROOT
for L in flink_amd/libgwo.so $(ls exp/libgwo_*.so 2>/dev/null); do
  GWO_LIB_PATH=$PWD/$L timeout -k 10 200 python bench.py --warmup ${W:-9} --steps ${S:-3} --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { echo FAIL $L; tail -5 gpurun_out/ab.log; exit 1; }
  echo $L; tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e9,2), round(d['ms_per_step'],3), {k: round(v['total_ms']/v['launches'],3) for k,v in d['kernels_ms'].items()})"
done
