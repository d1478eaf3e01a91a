# Round 6: C5 process-kernel ablations (timing only; results invalid): exp/norec (records loaded, not applied),
# exp/noend (no write-back), exp/noboth -- rocprofv3 --stats of bench_configs c5 per variant.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r06y
mkdir -p $O
export TMPDIR=/tmp
for L in exp/norec/libgwo.so exp/noend/libgwo.so exp/noboth/libgwo.so; do
  tag=$(echo $L | tr '/' '_'); lp=$R/$L; [ $L = product ] && lp=
  ( cd /tmp && GWO_LIB_PATH=$lp BENCH_PROF=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- python3 $R/bench_configs.py c5 > $O/$tag.log 2>&1 ) || { echo FAIL $L; tail $O/$tag.log; exit 1; }
  python3 - "$O/$tag/run_kernel_stats.csv" "$L" <<'PY'
import csv, sys
rows = {r['Name'].split('(')[0].split('::')[-1]: float(r['AverageNs']) / 1e3 for r in csv.DictReader(open(sys.argv[1]))}
print(sys.argv[2], {k: round(v, 1) for k, v in rows.items() if k.startswith('sess_')})
PY
done
