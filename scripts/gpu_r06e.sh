# Round 6: emit selection A/B (masks: product, vs exp/emitbr: per-row scalar branches), two rounds, then the full GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
VARIANTS="base emitbr base emitbr" bash scripts/gpu_ab.sh || exit 1
TEST_TIMEOUT=1000 PER_TEST=300 bash scripts/gpu_tests.sh
