# Per-kernel PMC counters of a short bench run: one rocprofv3 --pmc pass per counter group, each its
# own run (MI355X_MICROARCH.md: TCC slots -- FETCH_SIZE takes 3, WRITE_SIZE 2; gfx950 FETCH_SIZE
# reads half the bytes of wide coalesced streams).  PASSES overrides the groups (';'-separated).
set -o pipefail
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
PASSES=${PASSES:-"FETCH_SIZE;WRITE_SIZE"}
IFS=';' read -ra GROUPS_ <<< "$PASSES"
i=0
for C in "${GROUPS_[@]}"; do
  i=$((i+1))
  mkdir -p $R/gpurun_out/pmc_$i
  echo "pass $i: $C" > $R/gpurun_out/pmc_$i/counters.txt
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex "${KREGEX:-gwo}" --output-format csv -d $R/gpurun_out/pmc_$i -o run -- python3 $R/bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $R/gpurun_out/pmc_$i.log 2>&1 || { echo PMC_FAIL $C; tail -20 $R/gpurun_out/pmc_$i.log; exit 1; }
done
ls $R/gpurun_out/pmc_*
