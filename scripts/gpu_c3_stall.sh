# Where the C3 window step's waves wait: SQ activity, L2 write-back stalls, L1->L2 latencies (separate PMC passes over
# bench_configs.py c3; kernels matching slog_fire), and the same for the C4 bench's K1 and fire for comparison.
set -o pipefail
P="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU;TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_EA0_WRREQ_STALL_sum TCC_HIT_sum TCC_MISS_sum;TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum"
PYCMD="bench_configs.py c3" KREGEX="slog_fire" TAG=c3st PASSES="$P" bash scripts/gpu_pmc_py.sh && \
PYCMD="bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-host-fed" KREGEX="log_part|log_fire|log_split" TAG=c4st PASSES="$P" bash scripts/gpu_pmc_py.sh
