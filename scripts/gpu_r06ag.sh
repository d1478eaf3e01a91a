# Round 6: C5 host profile (GWO_SESS_HOST_PROF points inside insert_session / fire_session + per-call times).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06ag
for v in "" "GWO_SESS_FIRE_EVENT=1"; do
  env $v GWO_SESS_HOST_PROF=1 BENCH_PROF=0 BENCH_HOST_TIMING=1 timeout -k 10 200 python3 -u bench_configs.py c5 > gpurun_out/r06ag/c5_$v.log 2>&1 || exit 1
  echo "[$v]"; grep -E 'host us|session host' gpurun_out/r06ag/c5_$v.log; tail -n 1 gpurun_out/r06ag/c5_$v.log | cut -c1-200
done
