# Round 6 final validation 4 (after the gather tail change): the whole GPU suite, smoke(), the driver's bench
# command, and C2's roofline at this tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06final4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --durations=10 --timeout 200 --timeout-method thread \
    > $O/pytest_all.log 2>&1
rc=$?
tail -n 3 $O/pytest_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
tail -n 1 $O/bench.log | cut -c1-300
CONFIGS="c2" bash scripts/gpu_cfg_roofline.sh || exit 1
