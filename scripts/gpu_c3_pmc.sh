# C3 window step: phase trace (GWO_SLOG_TRACE) + slog_fire_kernel PMC passes (separate runs, per-block limits).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
GWO_SLOG_TRACE=1 timeout -k 10 240 python -u bench_configs.py c3 > gpurun_out/c3_slogtrace.log 2>&1 || { echo TRACE_FAIL; tail -20 gpurun_out/c3_slogtrace.log; exit 1; }
grep '^\[slog\]' gpurun_out/c3_slogtrace.log | head -4
tail -1 gpurun_out/c3_slogtrace.log | cut -c1-400
PYCMD="bench_configs.py c3" KREGEX="slog_fire" TAG=${TAG:-c3pmc} \
PASSES="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY;FETCH_SIZE;WRITE_SIZE" \
  bash scripts/gpu_pmc_py.sh
