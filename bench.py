#!/usr/bin/env python3
"""Headline benchmark: keyed event-time tumbling window aggregation, high-cardinality config C4.

Workload (BASELINE.json configs[3]): 100M int64 keys per GPU, tumbling 10 s
windows, sum/min/max over an int64 value, maxParallelism 32768, event time spanning 60 s with
U[0, 1 s) disorder and punctuated watermarks (lag 1 s) once per second of event time.  Per GPU the
stream is 1e9 records (16.7M per step); the input is generated into HBM before the timed region.

A "step" = one watermark interval: gwo_submit(batch) (classify + partition into the windows'
record logs) + gwo_advance_watermark (fire: fold every window whose end passed and
emit its rows).  The operator reserves its steady-state device memory at creation from the
distinct-keys hint, so any warmup >= 0 measures the steady state; 20 timed steps include two fires
(a window fires every 10 steps).  With --gpus N the job runs one process per GPU (under torch.distributed.run,
or spawned here when WORLD_SIZE is unset; fewer GPUs than N is an error); every rank generates
its own slice of a 100M*N-key stream and gwo_submit shuffles records to their key-group owner with an
RCCL all-to-all (weak scaling).

The roofline kernel is the one with the most time in the timed region.  K1 (log_part_kernel) times itself on
the device wall clock -- workgroup 0's start and its last workgroup's end, read back with its plan -- so the
timed region carries no stream markers between K1 and pass 2 (each costs the stream ~5 us: 1.3 % of a step);
the fire is bracketed by HIP events on the handle's stream (one window per 10 steps).  host_fed is a
separate, smaller run: pinned host columns in, fired rows drained to pinned host memory (PCIe-bound,
never the headline value).

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
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--records-per-gpu", type=int, default=1_000_000_000)
    p.add_argument("--keys-per-gpu", type=int, default=100_000_000)
    p.add_argument("--span-ms", type=int, default=60_000)
    p.add_argument("--window-ms", type=int, default=10_000)
    p.add_argument("--wm-interval-ms", type=int, default=1_000)
    p.add_argument("--lag-ms", type=int, default=1_000)
    p.add_argument("--max-parallelism", type=int, default=32768)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-scale", type=int, default=8,
                   help="CPU baseline sample: the C4 stream with keys and records per step divided by this")
    p.add_argument("--layout", choices=["auto", "log", "table"], default="auto",
                   help="device state layout (auto = the log layout at this cardinality)")
    p.add_argument("--no-host-fed", action="store_true")
    p.add_argument("--host-fed-steps", type=int, default=12)
    p.add_argument("--no-profile", action="store_true",
                   help="no per-kernel HIP events in the timed region (diagnostic: the events' own cost)")
    p.add_argument("--pipeline", action="store_true",
                   help="pipelined submission (gwo_set_pipelined_submit): measured slower on C4, since pass 2 then "
                        "runs after the next batch's K1 and misses its batch buffer in the MALL")
    p.add_argument("--sync-watermark", action="store_true",
                   help="multi-GPU: agree on each watermark synchronously (default: gwo_comm_set_async_watermark)")
    p.add_argument("--comm-single", action="store_true",
                   help="attach a 1-rank RCCL communicator at N=1 (one rank: no record leaves the GPU)")
    p.add_argument("--comm-virtual", type=int, default=0,
                   help="with --comm-single: route as GPU 0 of P GPUs (GWO_COMM_VIRTUAL=P), the other GPUs' records "
                        "through RCCL to this rank itself -- a rank's multi-GPU data path at P, measured on one GPU")
    return p.parse_args()


def host_cores():
    """Host cores this process may use: the CPU affinity mask, capped by a cgroup CPU quota (cpu.max) when one is
    set.  Returns (cores, detail)."""
    cpus = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = cpus
    quota = None
    for f in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            txt = open(f).read().split()
        except OSError:
            continue
        if f.endswith("cpu.max") and txt and txt[0] != "max":
            quota = int(txt[0]) / int(txt[1])
        elif f.endswith("cfs_quota_us") and txt and int(txt[0]) > 0:
            quota = int(txt[0]) / int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        break
    cores = aff if quota is None else max(1, min(aff, int(quota)))
    return cores, {"os_cpu_count": cpus, "affinity": aff, "cgroup_cpu_quota": quota}


def kfd_gpu_count(topology="/sys/class/kfd/kfd/topology/nodes"):
    """GPUs this process may use, from the KFD topology in sysfs (nodes with SIMDs are GPUs; the logic of
    tools/amd-gpu-discovery.sh), restricted by HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES
    when set.  No HIP call: the spawning parent must not initialise the GPU before its children start."""
    n = 0
    try:
        nodes = sorted((d for d in os.listdir(topology) if d.isdigit()), key=int)
    except OSError:
        nodes = []
    for d in nodes:
        try:
            for line in open(os.path.join(topology, d, "properties")):
                f = line.split()
                if len(f) == 2 and f[0] == "simd_count" and int(f[1]) > 0:
                    n += 1
                    break
        except (OSError, ValueError):
            continue
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def spawn_ranks(a):
    """--gpus N without a launcher: one child process per GPU (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set), as
    torch.distributed.run would start them.  This parent makes no GPU call (it counts devices in the KFD sysfs
    topology, not through HIP) and waits for the children; rank 0 prints the line."""
    import socket
    import subprocess
    have = kfd_gpu_count()
    if have < a.gpus:
        sys.exit(f"bench.py: --gpus {a.gpus} needs {a.gpus} GPUs, this host has {have}")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        rc = p.wait() or rc
    sys.exit(rc)


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        spawn_ranks(a)
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != a.gpus:
        sys.exit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}")
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
                             key_group_range=rng, device=local, expected_keys=exp_keys, state_layout=a.layout)
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
        if a.comm_virtual > 1:
            os.environ["GWO_COMM_VIRTUAL"] = str(a.comm_virtual)
        N.check(lib.gwo_comm_init(h, uid, 1, 0), h, "gwo_comm_init")
        os.environ.pop("GWO_COMM_VIRTUAL", None)
    has_comm = world > 1 or a.comm_single
    if has_comm and not a.sync_watermark:   # the watermark all-reduce is not waited for (applied one call later)
        N.check(lib.gwo_comm_set_async_watermark(h, 1), h, "async watermark")

    def comm_stats():
        v = [C.c_int64() for _ in range(3)]
        N.check(lib.gwo_comm_stats(h, *[C.byref(x) for x in v]), h, "gwo_comm_stats")
        return [x.value for x in v]

    # the per-step arguments are built before timing: a step is the operator's three calls
    kp, tp, vp = key.data_ptr(), ts.data_ptr(), val.data_ptr()
    args = [(C.c_void_p(kp + 8 * s), C.c_void_p(tp + 8 * s), C.c_void_p(vp + 8 * s), e - s, wms[i])
            for i, (s, e) in enumerate(bounds)]
    submit, advance, discard = lib.gwo_submit, lib.gwo_advance_watermark, lib.gwo_discard_output

    def step(i):
        a_ = args[i]
        # rows stay in HBM (discarded): the sink is not part of the path
        if submit(h, a_[0], a_[1], a_[2], a_[3]) or advance(h, a_[4]) or discard(h):
            N.check(lib.gwo_sync(h), h, "step")   # surfaces the handle's error message
            raise RuntimeError(f"step {i} failed")

    def rows_emitted():
        r = C.c_int64()
        N.check(lib.gwo_rows_emitted(h, C.byref(r)), h)
        return r.value

    for i in range(a.warmup):
        step(i)
    N.check(lib.gwo_sync(h), h)
    cs0 = comm_stats() if has_comm else None
    rows_before = rows_emitted()
    lib.gwo_reset_stats(h)
    # time K1 and the fire (the candidates for the dominant kernel); pass 2 is never dominant here
    lib.gwo_set_profiling_mask(h, 0 if a.no_profile else (1 << N.KERNEL_INSERT) | (1 << N.KERNEL_FIRE))
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
    comm = None
    if has_comm:   # host waits inside the timed steps (gwo_comm_stats), max over ranks
        cs1 = comm_stats()
        d = [b - a_ for a_, b in zip(cs0, cs1)]
        if dist:
            t = torch.tensor(d, dtype=torch.int64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            d = t.tolist()
        comm = {"routed_batches": d[0], "count_waits": d[1], "watermark_waits": d[2],
                "watermark_agreement": "sync" if a.sync_watermark else "async",
                "virtual_ranks": a.comm_virtual if world == 1 else None}

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
        "fire": ("log_fire_kernel", stats["fire"][2] * REC_B + rows * O_B),
    }
    if a.layout == "table":   # scan + insert + fire sweep
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
    tj = json.load(open(tfile)) if os.path.exists(tfile) else {}
    t = tj.get(dname)
    if t:
        traffic = t["hbm_bytes_per_launch"]
    # path-level measured bytes: every kernel of the timed region's PMC bytes per launch x its launches
    # in the timed region (K1 and its pass 2 once per batch, the fire once per window), over the elapsed time
    pmc_path = None
    if a.layout != "table" and all(k in tj for k in ("log_part_kernel", "log_split_kernel", "log_fire_kernel")):
        k1n, fires = stats["insert"][0], stats["fire"][0]
        parts = {"log_part_kernel": (tj["log_part_kernel"]["hbm_bytes_per_launch"], k1n),
                 "log_split_kernel": (tj["log_split_kernel"]["hbm_bytes_per_launch"], k1n),
                 "log_fire_kernel": (tj["log_fire_kernel"]["hbm_bytes_per_launch"], fires)}
        pb = sum(b * n for b, n in parts.values())
        pmc_path = {"bytes_per_step": pb / a.steps, "achieved": pb / elapsed / 1e9, "unit": "GB/s",
                    "frac": pb / elapsed / 1e9 / 8000.0,
                    "per_kernel": {k: {"bytes_per_launch": b, "launches": n} for k, (b, n) in parts.items()},
                    "measured_at": tj.get("_meta", {"head": "unstamped"})}

    op.close()
    del key, ts, val
    torch.cuda.empty_cache()
    host_fed = None
    if rank == 0 and world == 1 and not a.no_host_fed:
        host_fed = host_fed_run(a, F, N, lib, local, rec_per_step, exp_keys)
    out = None
    if rank == 0:
        cpu = None
        if not a.no_cpu_baseline and world == 1:   # rank 0 at N=1 only
            cpu = cpu_baseline(a, N, lib, local)
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
                       "keys_per_gpu": a.keys_per_gpu, "records_per_gpu": records,
                       "records_generated_per_gpu": n_gen, "stream_rate": f"{R} records per {span} ms per GPU",
                       "records_per_step_per_gpu": rec_per_step,
                       "window_ms": a.window_ms, "watermark_every_ms": a.wm_interval_ms, "lag_ms": a.lag_ms,
                       "max_parallelism": a.max_parallelism, "parallelism": f"keyBy over {world} GPU(s)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s",
                         "frac": achieved / peak, "traffic": traffic, "kernel": dname,
                         "alg_bytes_per_launch": dbytes / max(dl, 1), "avg_launch_ms": avg_ms,
                         "launches": dl, "traffic_source": "profiles/traffic.json (rocprofv3 PMC)" if traffic else None,
                         "traffic_measured_at": tj.get("_meta", {}).get("head", "unstamped") if traffic else None},
            "roofline_path": {"alg_bytes_per_step": path_bytes / a.steps,
                              "achieved": path_bytes / elapsed / 1e9, "unit": "GB/s",
                              "frac": path_bytes / elapsed / 1e9 / peak,
                              "distinct_entries_per_step": u_tot / a.steps, "fired_rows_per_step": rows / a.steps},
            "roofline_pmc_path": pmc_path,
            "kernels_ms": {k: {"launches": v[0], "total_ms": v[1]} for k, v in stats.items() if v[0]},
            "cpu_baseline": cpu,
            "host_fed": host_fed,
        }
        if comm:
            out["comm"] = comm
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def gen_stream(N, lib, local, seed, total, nkeys, span, n, first=0):
    import torch
    dev = torch.device("cuda", local)
    k = torch.empty(n, dtype=torch.int64, device=dev)
    t = torch.empty(n, dtype=torch.int64, device=dev)
    v = torch.empty(n, dtype=torch.int64, device=dev)
    spec = N.GwoGenSpec(seed, first, total, nkeys, span, 1000, 0, 1000, N.DTYPE_INT64, 0)
    N.check(lib.gwo_generate(C.byref(spec), n, k.data_ptr(), t.data_ptr(), v.data_ptr(), None, local), None,
            "gwo_generate")
    torch.cuda.synchronize()
    return k, t, v


def step_watermarks(ts_host, per, nsteps, lag):
    wms, run = [], -(1 << 63)
    for i in range(nsteps):
        run = max(run, int(ts_host[i * per:(i + 1) * per].max()))
        wms.append(run - lag - 1)
    return wms


def host_fed_run(a, F, N, lib, local, per, exp_keys):
    """End-to-end from host memory (SURVEY.md §8d 'host-fed'): the C4 stream's first host_fed_steps steps as
    pinned host columns; per step gwo_submit(host pointers: one H2D copy per column on the handle's stream)
    + gwo_advance_watermark + every fired row drained into pinned host columns.  Window [0, 10 s) fires
    at step 10, so 12 steps include one full fire (~81M rows)."""
    import torch
    steps = a.host_fed_steps
    n = per * steps
    k, t, v = gen_stream(N, lib, local, 42, a.records_per_gpu, a.keys_per_gpu, a.span_ms, n)
    hk, ht, hv = (x.cpu().pin_memory() for x in (k, t, v))
    del k, t, v
    torch.cuda.empty_cache()
    wms = step_watermarks(ht.numpy(), per, steps, a.lag_ms)
    agg = F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.MaxAggregate())
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(a.window_ms), agg, max_parallelism=a.max_parallelism,
                             device=local, expected_keys=exp_keys)
    h = op.handle
    cap = exp_keys + exp_keys // 8 + 4096
    outs = [torch.empty(cap, dtype=torch.int64).pin_memory() for _ in range(6)]
    o = N.GwoOut()
    o.key, o.start, o.end = outs[0].data_ptr(), outs[1].data_ptr(), outs[2].data_ptr()
    for i in range(3):
        o.result[i] = outs[3 + i].data_ptr()
    drained = 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        s = i * per
        N.check(lib.gwo_submit(h, C.c_void_p(hk.data_ptr() + 8 * s), C.c_void_p(ht.data_ptr() + 8 * s),
                               C.c_void_p(hv.data_ptr() + 8 * s), per), h, "submit")
        N.check(lib.gwo_advance_watermark(h, wms[i]), h, "watermark")
        while True:
            got = C.c_int64()
            N.check(lib.gwo_drain(h, C.byref(o), cap, C.byref(got)), h, "drain")
            drained += got.value
            if got.value < cap:
                break
    N.check(lib.gwo_sync(h), h)
    secs = time.perf_counter() - t0
    op.close()
    return {"value": n / secs, "unit": "records/s", "steps": steps, "records": n, "rows_drained": drained,
            "note": "pinned host key/ts/value columns in (H2D inside gwo_submit), fired rows drained to pinned "
                    "host columns; 1 GPU, same C4 stream and operator config"}


def cpu_baseline(a, N, lib, local):
    """The oracle's C restatement of WindowOperator (oracle/window_oracle.c: per-subtask heap hash map +
    deduplicated timer heap, one thread per usable host core (host_cores()) sharded by key group; kind 'port', not
    Flink -- no JDK here) on a
    bounded sample of the same workload: the C4 stream with keys and records per step scaled down by
    --cpu-scale (keys per record unchanged), 11 one-second steps -- window [0, 10 s) complete -- ending
    with the final Long.MAX_VALUE watermark, so every window fires and state reaches its steady size."""
    from oracle import cbaseline
    if not cbaseline.available():
        return None
    sc = max(1, a.cpu_scale)
    total, nkeys = a.records_per_gpu // sc, a.keys_per_gpu // sc
    per = total * a.wm_interval_ms // a.span_ms
    steps = a.window_ms // a.wm_interval_ms + 1
    k, t, v = gen_stream(N, lib, local, 42, total, nkeys, a.span_ms, per * steps)
    kh, th, vh = k.cpu().numpy(), t.cpu().numpy(), v.cpu().numpy()
    del k, t, v
    wms = step_watermarks(th, per, steps, a.lag_ms)
    batches = [((i + 1) * per, wms[i]) for i in range(steps)] + [(per * steps, (1 << 63) - 1)]
    threads, detail = host_cores()
    t0 = time.perf_counter()
    _, _, late = cbaseline.run_tumbling(kh, th, vh, batches, a.window_ms, threads=threads,
                                        max_par=a.max_parallelism, rows=False)
    secs = time.perf_counter() - t0
    n = per * steps
    return {"value": n / secs, "unit": "records/s", "cores": threads, "kind": "port", "seconds": secs,
            "cores_detail": dict(detail, rule="threads = the CPU affinity mask, capped by the cgroup CPU quota"),
            "sample": f"C4 stream scaled 1/{sc}: {nkeys} keys, {per} records per 1-s step, {steps} steps "
                      f"({n} records: window [0, {a.window_ms} ms) complete) then the final Long.MAX_VALUE "
                      f"watermark (every window fires); C restatement of WindowOperator (oracle/window_oracle.c), "
                      f"{threads} threads sharded by key group"}


if __name__ == "__main__":
    main()
