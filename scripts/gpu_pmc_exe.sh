# PMC passes of a standalone executable (EXE with ARGS): one rocprofv3 --pmc run per ';'-separated counter group.
set -o pipefail
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
IFS=';' read -ra GROUPS_ <<< "$PASSES"
i=0
for C in "${GROUPS_[@]}"; do
  i=$((i+1))
  mkdir -p $R/gpurun_out/xpmc_$i
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "${KREGEX:-gwo}" --output-format csv -d $R/gpurun_out/xpmc_$i -o run -- $R/$EXE $ARGS > $R/gpurun_out/xpmc_$i.log 2>&1 || { echo PMC_FAIL $C; tail -20 $R/gpurun_out/xpmc_$i.log; exit 1; }
done
mkdir -p $R/gpurun_out/xtrace
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/xtrace -o run -- $R/$EXE $ARGS > $R/gpurun_out/xtrace.log 2>&1
