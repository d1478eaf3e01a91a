#!/usr/bin/env python3
"""Headline benchmark: keyed event-time tumbling window aggregation, high-cardinality config C4.

Workload (BASELINE.json configs[3]): 100M int64 keys per GPU, tumbling 10 s
windows, sum/min/max over an int64 value, maxParallelism 32768, event time spanning 60 s with
U[0, 1 s) disorder and punctuated watermarks (lag 1 s) once per second of event time.  Per GPU the
stream is 1e9 records (16.7M per step); the input is generated into HBM before the timed region.

A "step" = one watermark interval: gwo_submit(batch) (classify + partition into the windows'
record logs) + gwo_advance_watermark (fire: fold every window whose end passed and
emit its rows).  The default warmup (12 steps) covers one full window lifecycle (first fire at step
10), so the timed steps are the engine's steady state (device pools warm, output sized); 20 timed
steps include two fires.  With --gpus N the job runs one process per GPU; every rank generates its
own slice of a 100M*N-key stream and gwo_submit shuffles records to their key-group owner with an
RCCL all-to-all (weak scaling).

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
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=12)   # one full window lifecycle: pools warm
    p.add_argument("--records-per-gpu", type=int, default=1_000_000_000)
    p.add_argument("--keys-per-gpu", type=int, default=100_000_000)
    p.add_argument("--span-ms", type=int, default=60_000)
    p.add_argument("--window-ms", type=int, default=10_000)
    p.add_argument("--wm-interval-ms", type=int, default=1_000)
    p.add_argument("--lag-ms", type=int, default=1_000)
    p.add_argument("--max-parallelism", type=int, default=32768)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-sample", type=int, default=2_000_000)
    p.add_argument("--no-profile", action="store_true",
                   help="no per-kernel HIP events in the timed region (diagnostic: the events' own cost)")
    p.add_argument("--pipeline", action="store_true",
                   help="pipelined submission (gwo_set_pipelined_submit): measured slower on C4, since pass 2 then "
                        "runs after the next batch's K1 and misses its batch buffer in the MALL")
    p.add_argument("--comm-single", action="store_true",
                   help="attach a 1-rank RCCL communicator at N=1 (measures the exchange path on one GPU)")
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
    # sizing hint = expected distinct keys per window: uniform keys, records_per_window draws
    rec_per_window = R * a.window_ms // span
    exp_keys = int(a.keys_per_gpu * (1.0 - np.exp(-rec_per_window / a.keys_per_gpu)))
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(a.window_ms), agg, max_parallelism=a.max_parallelism,
                             key_group_range=rng, device=local, expected_keys=exp_keys)
    h = op.handle
    if a.pipeline:   # K1 of batch i queues before batch i-1 resolves (gwo.h gwo_set_pipelined_submit)
        N.check(lib.gwo_set_pipelined_submit(h, 1), h)
    if world > 1:
        uid = (C.c_uint8 * N.COMM_ID_BYTES)()
        if rank == 0:
            N.check(lib.gwo_comm_unique_id(uid))
        t_uid = torch.tensor(list(bytes(uid)), dtype=torch.uint8, device=dev)
        dist.broadcast(t_uid, 0)
        uid = (C.c_uint8 * N.COMM_ID_BYTES)(*t_uid.cpu().tolist())
        N.check(lib.gwo_comm_init(h, uid, world, rank), h, "gwo_comm_init")
    elif a.comm_single:
        uid = (C.c_uint8 * N.COMM_ID_BYTES)()
        N.check(lib.gwo_comm_unique_id(uid))
        N.check(lib.gwo_comm_init(h, uid, 1, 0), h, "gwo_comm_init")

    def step(i):
        s, e = bounds[i]
        N.check(lib.gwo_submit(h, C.c_void_p(key.data_ptr() + 8 * s), C.c_void_p(ts.data_ptr() + 8 * s),
                               C.c_void_p(val.data_ptr() + 8 * s), e - s), h, "submit")
        N.check(lib.gwo_advance_watermark(h, wms[i]), h, "watermark")
        N.check(lib.gwo_discard_output(h), h)   # rows stay in HBM; the sink is not part of the path

    def rows_emitted():
        r = C.c_int64()
        N.check(lib.gwo_rows_emitted(h, C.byref(r)), h)
        return r.value

    for i in range(a.warmup):
        step(i)
    N.check(lib.gwo_sync(h), h)
    rows_before = rows_emitted()
    lib.gwo_reset_stats(h)
    lib.gwo_set_profiling(h, 0 if a.no_profile else 1)
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

    stats = {name: kstat(k) for name, k in (("scan", N.KERNEL_SCAN), ("insert", N.KERNEL_INSERT),
                                             ("fire", N.KERNEL_FIRE), ("partition", N.KERNEL_PARTITION),
                                             ("exchange", N.KERNEL_EXCHANGE))}
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

    # ---- algorithmic bytes ----
    # path:   B_alg = N*I + U*2S + F*(S+O); I = 24 B (key, ts, value), S = 40 B (key, window, sum, min,
    #         max), O = 48 B (key, start, end, sum, min, max), U = distinct (key, window) per batch,
    #         F = fired rows.
    # kernels (log layout, the C4 default): log_part reads I per record and appends 16 B per accepted
    #         (key, value); log_split moves 16 B in + 16 B out per logged record; log_fire reads the
    #         window's 16-B records and writes O per row.
    I_B, S_B, O_B, REC_B = 24, 40, 48, 16
    u_tot = 0
    if rank == 0:
        wnd = a.window_ms
        for i in range(a.warmup, nsteps):
            s, e = bounds[i]
            pair = key[s:e] * 64 + torch.div(ts[s:e], wnd, rounding_mode="floor")
            u_tot += int(torch.unique(pair).numel())
    rows = rows_emitted() - rows_before
    path_bytes = records * I_B + u_tot * 2 * S_B + rows * (S_B + O_B)
    kern = {
        "insert": ("log_part_kernel", records * (I_B + REC_B)),
        "partition": ("log_split_kernel", records * 2 * REC_B),
        "fire": ("log_fire_kernel", stats["fire"][2] * REC_B + rows * O_B),
    }
    if stats["partition"][0] == 0:   # table layout: scan + insert + fire sweep
        kern = {"insert": ("insert_direct_kernel", records * I_B + u_tot * 2 * 32),
                "fire": ("fire_kernel", stats["fire"][2] * 32 + rows * O_B)}
    dom = max(kern, key=lambda k: stats[k][1])
    dname, dbytes = kern[dom]
    dl, dms, _ = stats[dom]
    avg_ms = dms / max(dl, 1)
    achieved = dbytes / max(dl, 1) / (avg_ms / 1e3) / 1e9 if avg_ms > 0 else 0.0
    peak = 8000.0
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tfile):
        t = json.load(open(tfile)).get(dname)
        if t:
            traffic = t["hbm_bytes_per_launch"]

    out = None
    if rank == 0:
        cpu = None
        if not a.no_cpu_baseline:
            cpu = cpu_baseline(a, key, ts, val, bounds, wms)
        ms_per_step = elapsed / a.steps * 1e3
        out = {
            "metric": "records/sec per node, keyed window agg @1/2/4/8 GPU; % of HBM peak",
            "value": total_records / elapsed,
            "unit": "records/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_per_step,
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
                         "frac": achieved / peak, "traffic": traffic, "kernel": dname,
                         "alg_bytes_per_launch": dbytes / max(dl, 1), "avg_launch_ms": avg_ms,
                         "launches": dl, "traffic_source": "profiles/traffic.json (rocprofv3 PMC)" if traffic else None},
            "roofline_path": {"alg_bytes_per_step": path_bytes / a.steps,
                              "achieved": path_bytes / elapsed / 1e9, "unit": "GB/s",
                              "frac": path_bytes / elapsed / 1e9 / peak,
                              "distinct_entries_per_step": u_tot / a.steps, "fired_rows_per_step": rows / a.steps},
            "kernels_ms": {k: {"launches": v[0], "total_ms": v[1]} for k, v in stats.items() if v[0]},
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
