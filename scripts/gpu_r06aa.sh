# Round 6: C5 -- the session record function on LDS-typed lists (product) vs one flat-pointer path (exp/flat), each
# at 8 / 4 / 2 inline session slots (GWO_SESSION_SLOTS), 2 rounds; then the session tests on the product at 2 slots
# and at the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06aa
mkdir -p $O
for rep in 1 2; do
  for L in exp/flat/libgwo.so product; do
    for s in 8 4 2; do
      tag=$(echo $L | tr '/' '_')_s$s; lp=$L; [ $L = product ] && lp=
      GWO_LIB_PATH=$lp GWO_SESSION_SLOTS=$s BENCH_PROF=0 timeout -k 10 240 python3 -u bench_configs.py c5 > $O/$tag.$rep.log 2>&1 || { echo FAIL $tag; tail -20 $O/$tag.$rep.log; exit 1; }
      tail -n 1 $O/$tag.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L slots $s', 'ms/step %.4f' % d['ms_per_step'], 'G rec/s %.3f' % (d['value']/1e9))"
    done
  done
done
for s in 2 8; do
  GWO_SESSION_SLOTS=$s timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -k "sess or c5 or merging or multi_round or java or heap_state or checkpoint" --timeout 200 --timeout-method thread > $O/pytest_s$s.log 2>&1
  echo "slots=$s tests rc=$?"; tail -n 1 $O/pytest_s$s.log
done
