# Round 6 final measurement set for C4 (re-stamped at the final tree) (bench.py, the driver's configuration), one gpurun call:
#   1. rocprofv3 --kernel-trace --stats of bench.py --steps 20 --warmup 5
#   2. PMC FETCH_SIZE, WRITE_SIZE (separate runs) -> gpurun_out/r06at/traffic.json, stamped with TRAFFIC_HEAD, copied
#      to profiles/traffic.json on the box so that step 3 reports it
#   3. bench.py (default arguments: the driver's command) -> the bench line with roofline, traffic, cpu_baseline
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r06at
mkdir -p $O
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
    -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-fed > $O/prof_bench.log 2>&1 ) \
    || { echo PROF_FAIL; tail -20 $O/prof_bench.log; exit 1; }
tail -1 $O/prof_bench.log | cut -c1-300
rm -rf $R/gpurun_out/pmc_*
PASSES="FETCH_SIZE;WRITE_SIZE" KREGEX="log_" bash scripts/gpu_pmc.sh > $O/pmc.log 2>&1 || { echo PMC_FAIL; tail $O/pmc.log; exit 1; }
TRAFFIC_CMD="scripts/gpu_r06at.sh (gpu_pmc.sh FETCH_SIZE;WRITE_SIZE over bench.py --steps 10)" \
    python3 scripts/pmc_summary.py $R/gpurun_out $O/traffic.json > $O/pmc_summary.txt || exit 1
cp $O/traffic.json profiles/traffic.json
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value']/1e9, d['ms_per_step'], d['roofline']); print(d.get('cpu_baseline')); print(d.get('roofline_pmc_path'))"
