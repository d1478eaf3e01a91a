# Round 6: the session sweep on fire_stream overlapping the next batch's slot pass -- session parity tests first,
# then C5 A/B (exp/base/libgwo_s0.so = the same tree with the sweep on the handle's stream).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -v -x -k "sess or c5 or merging or java or heap_state or checkpoint or watermark" \
    --timeout 200 --timeout-method thread > $O/pytest_sess.log 2>&1
rc=$?
tail -6 $O/pytest_sess.log
[ $rc -eq 0 ] || exit $rc
LIBS="exp/base/libgwo_s0.so product" CFG=c5 REPS=3 bash scripts/gpu_cfg_ab.sh || exit 1
