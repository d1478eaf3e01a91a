# HBM traffic per kernel: separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE), each in its own run
# (MI355X_MICROARCH.md: TCC slots -- FETCH_SIZE takes 3, WRITE_SIZE 2; gfx950 FETCH_SIZE reads half
# the bytes of wide coalesced streams).
set -o pipefail
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  mkdir -p $R/gpurun_out/pmc_$C
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmc_$C -o run -- python3 $R/bench.py --steps ${STEPS:-4} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $R/gpurun_out/pmc_$C.log 2>&1 || { echo PMC_FAIL $C; tail -20 $R/gpurun_out/pmc_$C.log; exit 1; }
done
ls $R/gpurun_out/pmc_*
