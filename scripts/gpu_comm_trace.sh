# Kernel trace of the C4 bench at 8 virtual ranks (deferred receives), then the same bench with more RCCL p2p
# channels (the virtual ranks' self-sends are RCCL copy kernels).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ctrace
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ctrace -o run -- python3 $R/bench.py --steps 10 --warmup 8 --no-cpu-baseline --no-host-fed --comm-single --comm-virtual 8 > $R/gpurun_out/ctrace/bench.log 2>&1 || { echo TRACE_FAIL; tail -30 $R/gpurun_out/ctrace/bench.log; exit 1; }
tail -1 $R/gpurun_out/ctrace/bench.log | cut -c1-300
cd $R
for ch in 32; do
  NCCL_MIN_P2P_NCHANNELS=$ch NCCL_MIN_NCHANNELS=$ch timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-fed --comm-single --comm-virtual 8 > gpurun_out/ctrace/bench_ch$ch.log 2>&1 || { echo FAIL; tail -20 gpurun_out/ctrace/bench_ch$ch.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ctrace/bench_ch$ch.log').read().strip().splitlines()[-1]); print('ch$ch', round(d['value']/1e9,2), 'G rec/s', round(d['ms_per_step'],4), 'ms/step')"
done
