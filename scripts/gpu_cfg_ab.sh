# A/B of library variants on one bench_configs.py configuration within one GPU call: LIBS="path1 path2" (empty
# string entry = the product library; "env:A=1,B=0" = the product library under those variables), CFG (default c5),
# REPS rounds; each run under its own limit.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/cfgab
mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
  for L in ${LIBS:-product}; do
    tag=$(echo "$L" | tr '/' '_')
    lp=$L; [ "$L" = product ] && lp=
    ev=
    case "$L" in env:*) lp=; ev=$(echo "${L#env:}" | tr ',' ' ');; esac
    env $ev BENCH_PROF=${BENCH_PROF:-0} GWO_LIB_PATH=$lp timeout -k 10 240 python3 -u bench_configs.py ${CFG:-c5} \
        > $O/$tag.$rep.log 2>&1 || { echo "FAIL $L"; tail -20 $O/$tag.$rep.log; exit 1; }
    tail -n 1 $O/$tag.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L', 'ms/step %.4f' % d['ms_per_step'], 'G rec/s %.3f' % (d['value']/1e9))"
  done
done
