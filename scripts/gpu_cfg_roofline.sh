# Per-configuration rooflines (bench_configs.py --kernel-stats / --traffic), one gpurun call:
#   1. rocprofv3 --kernel-trace --stats of the configuration (one drive: BENCH_PROF=0) -> the kernel-stat CSV
#   2. rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE (separate runs) -> per-kernel HBM bytes per launch
#   3. the traffic of every configuration merged into gpurun_out/r06cfg/traffic_cfg.json (stamped with TRAFFIC_HEAD)
#   4. bench_configs.py cX --kernel-stats <CSV> --traffic <json> -> the configuration's JSON line
# Every GPU step under its own limit; the first failure ends the script.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r06cfg
mkdir -p $O
export TMPDIR=/tmp
CONFIGS=${CONFIGS:-c1 c2 c3 c5}
for c in $CONFIGS; do
  ( cd /tmp && BENCH_PROF=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$c -o run \
      -- python3 $R/bench_configs.py $c > $O/trace_$c.log 2>&1 ) || { echo "TRACE_FAIL $c"; tail -20 $O/trace_$c.log; exit 1; }
  i=0
  for C in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    ( cd /tmp && BENCH_PROF=0 timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "gwo" --output-format csv \
        -d $O/$c/pmc_$i -o run -- python3 $R/bench_configs.py $c > $O/pmc_${c}_$i.log 2>&1 ) || { echo "PMC_FAIL $c $C"; tail -20 $O/pmc_${c}_$i.log; exit 1; }
  done
  python3 scripts/pmc_summary.py $O/$c $O/traffic_$c.json > $O/pmc_${c}_summary.txt || exit 1
done
python3 - "$O" $CONFIGS <<'EOF' || exit 1
import json, sys, os
o, cfgs = sys.argv[1], sys.argv[2:]
merged = {}
for c in cfgs:
    t = json.load(open(os.path.join(o, f"traffic_{c}.json")))
    meta = t.pop("_meta", {})
    merged[c] = t
merged["_meta"] = dict(meta, command="scripts/gpu_cfg_roofline.sh (rocprofv3 --pmc FETCH_SIZE; WRITE_SIZE over "
                                     "BENCH_PROF=0 bench_configs.py cX)")
json.dump(merged, open(os.path.join(o, "traffic_cfg.json"), "w"), indent=1)
EOF
for c in $CONFIGS; do
  timeout -k 10 300 python3 bench_configs.py $c --kernel-stats $O/trace_$c/run_kernel_stats.csv \
      --traffic $O/traffic_cfg.json > $O/cfg_$c.json 2> $O/cfg_$c.err || { echo "CFG_FAIL $c"; tail -10 $O/cfg_$c.err; exit 1; }
  tail -1 $O/cfg_$c.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c', round(d['value']/1e9,3), 'G rec/s', r['kernel'], 'avg', r['avg_launch_ms'], 'frac', r['frac'], 'pmc_path', (d['roofline_pmc_path'] or {}).get('frac'))"
done
