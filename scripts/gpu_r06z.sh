# Round 6: C5 with fewer inline session slots per key entry (GWO_SESSION_SLOTS 2 / 4 / 8 = product default), 3 rounds;
# then the session tests at 4 slots.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06z
mkdir -p $O
for rep in 1 2 3; do
  for s in 8 4 2; do
    GWO_SESSION_SLOTS=$s BENCH_PROF=0 timeout -k 10 240 python3 -u bench_configs.py c5 > $O/s$s.$rep.log 2>&1 || { echo FAIL $s; tail -20 $O/s$s.$rep.log; exit 1; }
    tail -n 1 $O/s$s.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('slots $s', 'ms/step %.4f' % d['ms_per_step'], 'G rec/s %.3f' % (d['value']/1e9))"
  done
done
GWO_SESSION_SLOTS=4 timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -k "sess or c5 or merging or multi_round" --timeout 200 --timeout-method thread > $O/pytest_s4.log 2>&1
echo "slots=4 tests rc=$?"; tail -n 1 $O/pytest_s4.log
