# Round 6: C4 under the spin's stream-query interval: 500 us (product), 30 us (old cadence), 100 us; 3 rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfgab
for rep in 1 2 3; do
  for v in "GWO_SPIN_QUERY_US=500" "GWO_SPIN_QUERY_US=30" "GWO_SPIN_QUERY_US=100"; do
    env $v timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/cfgab/c4_$v.$rep.log 2>&1 || exit 1
    echo "C4 [$v] $(tail -n 1 gpurun_out/cfgab/c4_$v.$rep.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
