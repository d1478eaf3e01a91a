# rocprofv3 kernel-trace of bench_configs.py CFG (default c5) per library variant (VARIANTS; base = flink_amd/libgwo.so):
# per-kernel average durations side by side.
set -o pipefail
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then L=""; else L=$R/exp/$v/libgwo.so; fi
  mkdir -p $R/gpurun_out/pab_$v
  GWO_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pab_$v -o run -- python3 $R/bench_configs.py ${CFG:-c5} > $R/gpurun_out/pab_$v/bench.log 2>&1 || { echo FAIL $v; tail -5 $R/gpurun_out/pab_$v/bench.log; exit 1; }
  python3 - $R/gpurun_out/pab_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[2], ' '.join('%s=%.1f' % (r['Name'].split('(')[0].replace('void ', '').replace('gwo::', '')[:24], float(r['AverageNs']) / 1e3) for r in rows[:6]))
PY
done
