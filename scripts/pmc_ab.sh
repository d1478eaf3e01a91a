# SQ counters of the fire kernel, new library vs libgwo_old.so (A/B).  Output: gpurun_out/pmc_{new,old}/
set -o pipefail
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
C="${PMC:-SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY}"
for v in new old; do
  mkdir -p $R/gpurun_out/pmcab_$v/pmc_1
  LIBP=""
  [ $v = old ] && export GWO_LIB_PATH=$R/flink_amd/libgwo_old.so
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex log_fire --output-format csv -d $R/gpurun_out/pmcab_$v/pmc_1 -o run -- python3 $R/bench.py --steps 12 --warmup 2 --no-cpu-baseline > $R/gpurun_out/pmcab_$v.log 2>&1 || { echo PMC_FAIL $v; tail -20 $R/gpurun_out/pmcab_$v.log; exit 1; }
  echo "== $v"; python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmcab_$v
done
unset GWO_LIB_PATH
