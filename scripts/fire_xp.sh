# Fire-kernel ablation: bench.py under GWO_FIRE_XP variants (1 = no row stores, 2 = no row-counter
# atomic, 4 = no fold, 8 = claim phase only, 16 = per-phase clock64 printout of workgroup 0,
# 32 = drain memory before each partition).  Output: gpurun_out/xp_<v>.log
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in ${XPS:-0 1 2 4 8}; do
  GWO_LIB_PATH=${LIBP:-} GWO_FIRE_XP=$v timeout -k 10 120 python -u bench.py --steps 20 --warmup 12 --no-cpu-baseline > gpurun_out/xp_$v.log 2>&1 || { echo FAIL $v; tail -5 gpurun_out/xp_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/xp_$v.log').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],4), {k:round(v['total_ms']/v['launches'],4) for k,v in d['kernels_ms'].items()})"
  grep FIREPROF gpurun_out/xp_$v.log | tail -2 || true
done
