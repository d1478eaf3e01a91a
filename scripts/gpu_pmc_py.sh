# PMC passes over a python command (PYCMD), kernels matching KREGEX: one rocprofv3 --pmc run per ';'-separated
# counter group (each group within the per-block limits), results under gpurun_out/ppmc_<i>/.
set -o pipefail
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
IFS=';' read -ra GROUPS_ <<< "$PASSES"
i=0
for C in "${GROUPS_[@]}"; do
  i=$((i+1))
  mkdir -p $R/gpurun_out/${TAG:-ppmc}_$i
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex "${KREGEX:-gwo}" --output-format csv -d $R/gpurun_out/${TAG:-ppmc}_$i -o run -- python3 $R/$PYCMD > $R/gpurun_out/${TAG:-ppmc}_$i.log 2>&1 || { echo PMC_FAIL $C; tail -20 $R/gpurun_out/${TAG:-ppmc}_$i.log; exit 1; }
  echo "pass $i done: $C"
done
