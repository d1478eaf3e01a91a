# Round 6: C5 process-kernel wave-cycle counters (one rocprofv3 --pmc pass) on the product (2 inline slots).
set -o pipefail
cd $GRAFT_REPO_ROOT
PASSES="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_WAIT_INST_LDS,SQ_INSTS_LDS,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_WAVES" \
  KREGEX="sess_" TAG=sesspmc PYCMD="bench_configs.py c5" BENCH_PROF=0 bash scripts/gpu_pmc_py.sh || exit 1
