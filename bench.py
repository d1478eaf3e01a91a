#!/usr/bin/env python3
"""Headline benchmark: keyed event-time tumbling window aggregation, high-cardinality config C4.

Workload (BASELINE.json configs[3]): 100M int64 keys per GPU, tumbling 10 s
windows, sum/min/max over an int64 value, maxParallelism 32768, event time spanning 60 s with
U[0, 1 s) disorder and punctuated watermarks (lag 1 s) once per second of event time.  Per GPU the
stream is 1e9 records (16.7M per step); the input is generated into HBM before the timed region.

A "step" = one watermark interval: gwo_submit(batch) (scan + insert into the per-window HBM
tables) + gwo_advance_watermark (fire kernels emit every window whose end passed).  With --gpus N
the job runs one process per GPU; every rank generates its own slice of a 100M*N-key stream and
gwo_submit shuffles records to their key-group owner with an RCCL all-to-all (weak scaling).

Prints ONE JSON line (rank 0).
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--records-per-gpu", type=int, default=1_000_000_000)
    p.add_argument("--keys-per-gpu", type=int, default=100_000_000)
    p.add_argument("--span-ms", type=int, default=60_000)
    p.add_argument("--window-ms", type=int, default=10_000)
    p.add_argument("--wm-interval-ms", type=int, default=1_000)
    p.add_argument("--lag-ms", type=int, default=1_000)
    p.add_argument("--max-parallelism", type=int, default=32768)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-sample", type=int, default=2_000_000)
    return p.parse_args()


def main():
    a = parse()
    import torch
    import flink_amd as F
    from flink_amd import _native as N

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    lib = N.lib()

    R = a.records_per_gpu
    span = a.span_ms
    rec_per_step = R * a.wm_interval_ms // span
    nsteps = a.warmup + a.steps
    if nsteps * a.wm_interval_ms > span:  # extend event time beyond 60 s (same rate) if asked for more steps
        span = nsteps * a.wm_interval_ms
        R = rec_per_step * nsteps
    n_gen = rec_per_step * nsteps
    nkeys = a.keys_per_gpu * world

    # ---- synthetic input, resident in HBM (untimed) ----
    dev = torch.device("cuda", local)
    key = torch.empty(n_gen, dtype=torch.int64, device=dev)
    ts = torch.empty(n_gen, dtype=torch.int64, device=dev)
    val = torch.empty(n_gen, dtype=torch.int64, device=dev)
    first = rank * R  # each rank generates its own slice of the global stream
    spec = N.GwoGenSpec(42, first, R, nkeys, span, 1000, 0, 1000, N.DTYPE_INT64, 0)
    # the rank's slice keeps the same event-time span: generate with a rank-local index base
    spec.first_index = 0
    spec.seed = 42 + 1_000_003 * rank
    N.check(lib.gwo_generate(C.byref(spec), n_gen, key.data_ptr(), ts.data_ptr(), val.data_ptr(), None, local),
            None, "gwo_generate")
    torch.cuda.synchronize()
    bounds = [(i * rec_per_step, (i + 1) * rec_per_step) for i in range(nsteps)]
    ts_cpu_max = [int(ts[s:e].max().item()) for s, e in bounds]  # running max per batch boundary
    wms = []
    run = -(1 << 63)
    for m in ts_cpu_max:
        run = max(run, m)
        wms.append(run - a.lag_ms - 1)

    # ---- operator ----
    if world > 1:
        kgr = F.compute_key_group_range_for_operator_index(a.max_parallelism, world, rank)
        rng = (kgr.start_key_group, kgr.end_key_group)
    else:
        rng = (0, a.max_parallelism - 1)
    agg = F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.MaxAggregate())
    exp_keys = int(a.keys_per_gpu * 0.9)
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(a.window_ms), agg, max_parallelism=a.max_parallelism,
                             key_group_range=rng, device=local, expected_keys=exp_keys)
    h = op.handle
    if world > 1:
        uid = (C.c_uint8 * N.COMM_ID_BYTES)()
        if rank == 0:
            N.check(lib.gwo_comm_unique_id(uid))
        t_uid = torch.tensor(list(bytes(uid)), dtype=torch.uint8, device=dev)
        dist.broadcast(t_uid, 0)
        uid = (C.c_uint8 * N.COMM_ID_BYTES)(*t_uid.cpu().tolist())
        N.check(lib.gwo_comm_init(h, uid, world, rank), h, "gwo_comm_init")

    def step(i):
        s, e = bounds[i]
        N.check(lib.gwo_submit(h, C.c_void_p(key.data_ptr() + 8 * s), C.c_void_p(ts.data_ptr() + 8 * s),
                               C.c_void_p(val.data_ptr() + 8 * s), e - s), h, "submit")
        N.check(lib.gwo_advance_watermark(h, wms[i]), h, "watermark")
        N.check(lib.gwo_discard_output(h), h)   # rows stay in HBM; the sink is not part of the path

    for i in range(a.warmup):
        step(i)
    N.check(lib.gwo_sync(h), h)
    lib.gwo_reset_stats(h)
    lib.gwo_set_profiling(h, 1)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.warmup, nsteps):
        step(i)
    N.check(lib.gwo_sync(h), h)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = t1 - t0
    lib.gwo_set_profiling(h, 0)

    def kstat(k):
        la, ms, it = C.c_int64(), C.c_double(), C.c_int64()
        lib.gwo_kernel_stats(h, k, C.byref(la), C.byref(ms), C.byref(it))
        return la.value, ms.value, it.value

    ins = kstat(N.KERNEL_INSERT)
    fire = kstat(N.KERNEL_FIRE)
    scan = kstat(N.KERNEL_SCAN)
    records = (nsteps - a.warmup) * rec_per_step
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
        r = torch.tensor([records], dtype=torch.float64, device=dev)
        dist.all_reduce(r)
        total_records = int(r.item())
    else:
        total_records = records

    # ---- roofline of the dominant kernel (insert): algorithmic bytes per launch ----
    # B_alg(insert) = n*I + U*2*S per launch; I = 24 B (key, ts, value), S = 32 B (key + sum/min/max;
    # the window start is implicit in the per-window table), U = distinct (key, window) per batch.
    I_B, S_B, O_B = 24, 32, 48
    u_tot = 0
    if rank == 0:
        wnd = a.window_ms
        for i in range(a.warmup, nsteps):
            s, e = bounds[i]
            pair = key[s:e] * 64 + torch.div(ts[s:e], wnd, rounding_mode="floor")
            u_tot += int(torch.unique(pair).numel())
    ins_launches, ins_ms, _ = ins
    fire_launches, fire_ms, fire_slots = fire
    alg_insert = (records * I_B + u_tot * 2 * S_B) / max(ins_launches, 1)
    avg_ins_s = ins_ms / max(ins_launches, 1) / 1e3
    achieved = alg_insert / avg_ins_s / 1e9 if avg_ins_s > 0 else 0.0
    peak = 8000.0

    out = None
    if rank == 0:
        cpu = None
        if not a.no_cpu_baseline:
            cpu = cpu_baseline(a, key, ts, val, bounds, wms)
        out = {
            "metric": "records/sec per node, keyed window agg @1/2/4/8 GPU; % of HBM peak",
            "value": total_records / elapsed,
            "unit": "records/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (splitmix64 counter generator, generated in HBM before timing)",
            "config": {"workload": "C4 high-cardinality tumbling sum/min/max",
                       "keys_per_gpu": a.keys_per_gpu, "records_per_gpu": R, "records_per_step_per_gpu": rec_per_step,
                       "window_ms": a.window_ms, "watermark_every_ms": a.wm_interval_ms, "lag_ms": a.lag_ms,
                       "max_parallelism": a.max_parallelism, "parallelism": f"keyBy over {world} GPU(s)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s",
                         "frac": achieved / peak, "traffic": None, "kernel": "insert_direct_kernel",
                         "alg_bytes_per_launch": alg_insert, "avg_launch_ms": avg_ins_s * 1e3,
                         "distinct_entries_per_launch": u_tot / max(ins_launches, 1)},
            "kernels_ms": {"scan": scan[1], "insert": ins_ms, "fire": fire_ms,
                           "fire_launches": fire_launches, "fire_slots": fire_slots},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    op.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def cpu_baseline(a, key, ts, val, bounds, wms):
    """Times the oracle's C restatement (oracle/_ref-free; kind 'port') on a bounded sample of the
    same workload on host cores; falls back to the numpy restatement when the C build is absent."""
    n = min(a.cpu_sample, bounds[-1][1])
    k = key[:n].cpu().numpy()
    t = ts[:n].cpu().numpy()
    v = val[:n].cpu().numpy()
    per = bounds[0][1] - bounds[0][0]
    batches = [(min((i + 1) * per, n), wms[i]) for i in range((n + per - 1) // per)]
    batches[-1] = (n, batches[-1][1])
    from oracle import cbaseline
    if cbaseline.available():
        threads = min(os.cpu_count() or 1, 16)
        secs = cbaseline.time_tumbling(k, t, v, batches, a.window_ms, threads)
        return {"value": n / secs, "unit": "records/s", "cores": threads, "kind": "port",
                "sample": f"first {n} records of the same C4 stream, same windows/watermarks; C restatement "
                          f"of WindowOperator (oracle/window_oracle.c), {threads} threads sharded by key group"}
    from oracle import vectorized as V
    t0 = time.perf_counter()
    V.tumbling_lateness0(k, t, v, batches, a.window_ms, 0, [1, 2, 3])
    secs = time.perf_counter() - t0
    return {"value": n / secs, "unit": "records/s", "cores": 1, "kind": "port",
            "sample": f"first {n} records; numpy restatement (oracle/vectorized.py), 1 thread"}


if __name__ == "__main__":
    main()
