# Bench with and without a 1-rank RCCL communicator: the exchange path's cost on one GPU.
cd $GRAFT_REPO_ROOT
for f in "" "--comm-single"; do
  timeout -k 10 200 python bench.py --warmup 12 --steps 10 --no-cpu-baseline $f > gpurun_out/cc.log 2>&1 || { echo FAIL; tail -5 gpurun_out/cc.log; exit 1; }
  tail -1 gpurun_out/cc.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e9,2), round(d['ms_per_step'],3), {k: round(v['total_ms']/v['launches'],3) for k,v in d['kernels_ms'].items()})"
done
