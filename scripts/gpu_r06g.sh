# Round 6: C5 A/B (the session sort/gather sizing, exp/base = before), then the log fire's LDS counters on C4.
set -o pipefail
cd $GRAFT_REPO_ROOT
LIBS="exp/base/libgwo.so product" CFG=c5 REPS=2 bash scripts/gpu_cfg_ab.sh || exit 1
PASSES="SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_LDS,SQ_INSTS_VALU,SQ_WAVES,SQ_BUSY_CYCLES,SQ_INSTS_SALU" \
  KREGEX="log_fire" TAG=firepmc PYCMD="bench.py --steps 10 --warmup 2 --no-host-fed --no-cpu-baseline" \
  bash scripts/gpu_pmc_py.sh || exit 1
