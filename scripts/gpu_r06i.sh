# Round 6: the full GPU suite on the session sweep beside the next slot pass and the combine path's gather beside the
# previous merge, then C5 / C2 A/B of both (env toggles GWO_SESS_SIDE_SWEEP, GWO_CB_OVERLAP), 2 rounds each.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --durations=10 --timeout 200 --timeout-method thread \
    > $O/pytest_all.log 2>&1
rc=$?
tail -6 $O/pytest_all.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for e in "GWO_SESS_SIDE_SWEEP=0 c5" "GWO_SESS_SIDE_SWEEP=1 c5" "GWO_CB_OVERLAP=0 c2" "GWO_CB_OVERLAP=1 c2"; do
    set -- $e
    env $1 BENCH_PROF=0 timeout -k 10 240 python3 -u bench_configs.py $2 > $O/ab_$1_$2.$rep.log 2>&1 || { echo "FAIL $e"; tail -20 $O/ab_$1_$2.$rep.log; exit 1; }
    tail -n 1 $O/ab_$1_$2.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$e', 'ms/step %.4f' % d['ms_per_step'], 'G rec/s %.3f' % (d['value']/1e9))"
  done
done
