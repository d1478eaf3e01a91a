#!/usr/bin/env python3
"""Throughput of the other BASELINE.json configurations (bench.py is the C4 headline).

  c1  README-style tumbling sum: 1M records, 10K Long keys, 5 s windows, watermark every 10K records
  c2  YSB-shaped: 10 s tumbling count per campaign (1K campaigns from 10K ad ids), 100M events at
      1M events/s of event time, watermark every second (the ad-event filter is not modelled)
  c3  sliding 60 s / 1 s average over 10M keys, 200M records over 120 s (pane design)
  c5  event-time sessions, 30 s gap: 100K keys, 10M records in bursts, arrival order = ts + U[0, 5 s),
      watermark maxTs - 5 s - 1 after every 10 s of event time

Inputs are synthetic and resident in HBM before timing (C5's stream is built on the host with numpy
and uploaded once).  A step = gwo_submit(batch) + gwo_advance_watermark + discarding the rows.
Prints one JSON line per configuration (same fields as bench.py; `roofline_path` uses SURVEY.md
§8d's B_alg with the configuration's I/S/O).  Usage: python bench_configs.py [c1 c2 c3 c5]
  [--kernel-stats CSV] [--traffic JSON]

`roofline` is the dominant kernel's (the one with the most time in a rocprofv3 kernel trace of the same
configuration): its algorithmic bytes per launch (DOMINANT below: the bytes the reference's per-record work
must move, per launch) over its average launch time from `--kernel-stats` (the rocprofv3 `--stats` CSV of
`BENCH_PROF=0 python bench_configs.py cX`), against the 8 TB/s HBM peak; `traffic` and `roofline_pmc_path`
come from `--traffic` (profiles/traffic_cfg.json: rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE per launch and
configuration, scripts/pmc_summary.py, stamped with the source tree it was measured on).  Without the files
those fields are null.
"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

KERNELS = ("scan", "insert", "fire", "partition", "exchange", "slide", "session")

# Dominant kernel per configuration (rocprofv3 kernel traces, profiles/r05_final_cfg_c*_kernel_stats.csv and r06) and
# its algorithmic bytes per launch (SURVEY.md §8d units):
#   c1 scan_kernel: one batch's key + timestamp columns, 16 B per record (classification, key groups, statistics)
#   c2 gather_kernel: one batch's key + timestamp columns (COUNT reads no value), 16 B per record
#   c3 slog_fire_kernel: one window step -- the running total R read and R' written (key, 2 words, table slot: 26 B
#      per live key), the entering and the leaving pane's 16-B records, and one 32-B row (key, start, end, avg) per key
#   c5 sess_process_kernel: one batch's records (24 B) and one read + one write of each touched key's entry (the
#      table entry's header and inline session: 2 x 32 B per distinct key of the batch)
DOMINANT = {"c1": "scan_kernel", "c2": "gather_kernel", "c3": "slog_fire_kernel", "c5": "sess_process_kernel"}


def kernel_avg_ns(csv_path, name):
    """(calls, average ns) of the kernel `name` (the function name, template arguments aside) in a rocprofv3 --stats
    CSV; the instance with the most total time when several match."""
    import csv
    best = None
    for r in csv.DictReader(open(csv_path)):
        fn = r["Name"].split("(")[0].split("<")[0].split("::")[-1].replace("void ", "").strip()
        if fn == name and (best is None or float(r["TotalDurationNs"]) > float(best["TotalDurationNs"])):
            best = r
    return (int(best["Calls"]), float(best["AverageNs"])) if best else (0, None)


def kernel_calls(csv_path):
    import csv
    out = {}
    for r in csv.DictReader(open(csv_path)):
        fn = r["Name"].split("(")[0].split("<")[0].split("::")[-1].replace("void ", "").strip()
        out[fn] = out.get(fn, 0) + int(r["Calls"])
    return out


def gen_device(N, lib, dev, torch, n, nkeys, span, disorder, key_mode=0, seed=42):
    key = torch.empty(n, dtype=torch.int64, device=dev)
    ts = torch.empty(n, dtype=torch.int64, device=dev)
    val = torch.empty(n, dtype=torch.int64, device=dev)
    spec = N.GwoGenSpec(seed, 0, n, nkeys, span, disorder, 0, 1000, N.DTYPE_INT64, key_mode)
    N.check(lib.gwo_generate(C.byref(spec), n, key.data_ptr(), ts.data_ptr(), val.data_ptr(), None, 0), None, "gen")
    torch.cuda.synchronize()
    return key, ts, val


def session_stream(num_keys, n, gap=30_000, lag=5_000, seed=42, mean_inner=5_000, events_per_session=10):
    """Bursts per key with exponential inner gaps (< gap), separated by >= gap + 1 ms; arrival order
    sorted by ts + U[0, lag) (same shape as SURVEY.md §8d's C5 generator)."""
    rng = np.random.default_rng(seed)
    per = max(1, n // num_keys)
    keys = np.repeat(np.arange(num_keys, dtype=np.int64), per)
    m = len(keys)
    inner = np.minimum(rng.exponential(mean_inner, m), gap - 1).astype(np.int64)
    new = rng.random(m) < 1.0 / events_per_session
    between = (gap + 1 + rng.exponential(gap, m)).astype(np.int64)
    step = np.where(new, between, inner)
    first = np.arange(m) % per == 0
    start = rng.integers(0, 60_000, num_keys)
    step[first] = 0
    ts = np.cumsum(step)
    ts = ts - np.repeat(ts[first], per) + np.repeat(start, per)
    vals = rng.integers(0, 1000, m).astype(np.int64)
    order = np.argsort(ts + rng.integers(0, lag, m), kind="stable")
    return keys[order], ts[order], vals[order]


def run(cfg, kernel_stats=None, traffic=None):
    import torch
    import flink_amd as F
    from flink_amd import _native as N
    lib = N.lib()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    lag = 1000
    if cfg == "c1":
        n, nkeys, span, every = 1_000_000, 10_000, 60_000, 10_000
        key, ts, val = gen_device(N, lib, dev, torch, n, nkeys, span, 1000)
        assigner, agg, exp = F.TumblingEventTimeWindows.of(5000), F.SumAggregate(), 0
        I_B, S_B, O_B, workload = 24, 24, 32, "C1 tumbling 5 s sum, 1M records, 10K keys"
    elif cfg == "c2":
        n, nkeys, span, every = 100_000_000, 1_000, 100_000, 1_000_000
        key, ts, val = gen_device(N, lib, dev, torch, n, nkeys, span, 1000, key_mode=1)
        assigner, agg, exp = F.TumblingEventTimeWindows.of(10_000), F.CountAggregate(), 1000
        I_B, S_B, O_B, workload = 16, 24, 32, "C2 YSB-shaped 10 s tumbling count per campaign, 1K campaigns"
    elif cfg == "c3":
        n, nkeys, span = 200_000_000, 10_000_000, 120_000
        every = n * 1000 // span
        key, ts, val = gen_device(N, lib, dev, torch, n, nkeys, span, 1000)
        assigner, agg, exp = F.SlidingEventTimeWindows.of(60_000, 1000), F.AverageAggregate(), nkeys
        I_B, S_B, O_B, workload = 24, 32, 32, "C3 sliding 60 s / 1 s avg, 10M keys, 200M records"
    elif cfg == "c5":
        lag = 5000
        k, t, v = session_stream(100_000, 10_000_000, lag=lag)
        n, every = len(k), 100_000
        key, ts, val = (torch.from_numpy(x).to(dev) for x in (k, t, v))
        assigner, agg, exp = F.EventTimeSessionWindows.withGap(30_000), F.SumAggregate(), 100_000
        I_B, S_B, O_B, workload = 24, 32, 32, "C5 event-time sessions 30 s gap, 100K keys, 10M records"
    else:
        raise SystemExit(f"unknown config {cfg}")
    if cfg == "c5":
        # punctuate by event time (every 10 s of the running max timestamp), as a periodic
        # BoundedOutOfOrderness generator would: the stream's sparse tail would otherwise put many
        # sessions of one key into a single batch ahead of its watermark
        rm = np.maximum.accumulate(t)
        cuts = np.flatnonzero(np.diff(rm // 10_000)) + 1
        edges = [0] + cuts.tolist() + [n]
        bounds = [(a, b) for a, b in zip(edges[:-1], edges[1:]) if b > a]
    else:
        bounds = [(s, min(s + every, n)) for s in range(0, n, every)]
    run_max, wms = -(1 << 63), []
    tsc = ts.cpu().numpy()
    for s, e in bounds:
        run_max = max(run_max, int(tsc[s:e].max()))
        wms.append(run_max - lag - 1)
    # the per-step arguments are built before timing: the loop is the operator's three calls per step
    kp, tp, vp = key.data_ptr(), ts.data_ptr(), val.data_ptr()
    args = [(C.c_void_p(kp + 8 * s), C.c_void_p(tp + 8 * s), C.c_void_p(vp + 8 * s), e - s, wms[i])
            for i, (s, e) in enumerate(bounds)]
    submit, advance, discard = lib.gwo_submit, lib.gwo_advance_watermark, lib.gwo_discard_output
    warm = max(1, len(bounds) // 10)
    # pipelined submission on the combine path (C2) and sessions (C5); C1's 10K-record batches measured slower with it
    # (36.4 vs 33.7 us/step: the adaptive pre-aggregation probe batches get redone)
    pipe = os.environ.get("BENCH_PIPE", "1" if cfg in ("c2", "c5") else "0") != "0"
    host_timing = os.environ.get("BENCH_HOST_TIMING", "0") != "0"

    def drive(prof):
        """One operator over the whole stream: `warm` untimed steps, then the rest timed.  prof: per-kernel HIP
        events (two stream markers per launch, several microseconds each) -- the kernel breakdown comes from a
        profiled pass of its own, so the timed value carries no markers."""
        op = F.GpuWindowOperator(assigner, agg, max_parallelism=128, expected_keys=exp)
        h = op.handle
        if pipe:   # gwo_set_pipelined_submit: batch i's kernels queue before batch i-1's readback is read
            N.check(lib.gwo_set_pipelined_submit(h, 1), h)

        def step(i):
            a = args[i]
            if submit(h, a[0], a[1], a[2], a[3]) or advance(h, a[4]) or discard(h):
                N.check(lib.gwo_sync(h), h, "step")            # surfaces the handle's error message
                raise RuntimeError(f"step {i} failed")

        def emitted():
            r = C.c_int64()
            N.check(lib.gwo_rows_emitted(h, C.byref(r)), h)
            return r.value

        for i in range(warm):
            step(i)
        N.check(lib.gwo_sync(h), h)
        rows0 = emitted()
        lib.gwo_reset_stats(h)
        lib.gwo_set_profiling(h, 1 if prof else 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if host_timing and not prof:   # BENCH_HOST_TIMING=1: each call's host time (diagnostics, stderr)
            ns = np.zeros((len(bounds) - warm, 3), dtype=np.int64)
            pc = time.perf_counter_ns
            for r, i in enumerate(range(warm, len(bounds))):
                a = args[i]
                c0 = pc()
                submit(h, a[0], a[1], a[2], a[3])
                c1 = pc()
                advance(h, a[4])
                c2 = pc()
                discard(h)
                ns[r] = (c1 - c0, c2 - c1, pc() - c2)
            med = np.median(ns, axis=0) / 1e3
            print(f"host us per call (median) submit {med[0]:.2f} advance {med[1]:.2f} discard {med[2]:.2f}; "
                  f"mean {ns.mean(axis=0) / 1e3}", file=sys.stderr)
        else:
            for i in range(warm, len(bounds)):
                step(i)
        N.check(lib.gwo_sync(h), h)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0

        def kstat(k):
            la, ms, it = C.c_int64(), C.c_double(), C.c_int64()
            lib.gwo_kernel_stats(h, k, C.byref(la), C.byref(ms), C.byref(it))
            return la.value, ms.value

        stats = {name: kstat(i) for i, name in enumerate(KERNELS)}
        rows_all = emitted()
        rows = rows_all - rows0
        op.close()
        return elapsed, rows, stats, rows_all

    elapsed, nrows, _, nrows_all = drive(False)
    prof_elapsed, _, stats, _ = drive(True) if os.environ.get("BENCH_PROF", "1") != "0" else (None, None, {}, None)
    rows = [nrows]
    recs = bounds[-1][1] - bounds[warm][0]
    path_bytes = recs * I_B + rows[0] * (S_B + O_B)   # U*2S omitted: not measured here (lower bound)
    steps_all = len(bounds)

    # ---- the dominant kernel's roofline (DOMINANT): algorithmic bytes per launch over the traced average ----
    # (averaged over every step of the drive, warm-up included, as the trace's launch average is: one launch per step)
    dname = DOMINANT[cfg]
    per_batch = [e - s for s, e in bounds]
    if cfg in ("c1", "c2"):
        alg = 16.0 * sum(per_batch) / len(per_batch)
        unit = "one batch: 16 B (key, timestamp) per record"
    elif cfg == "c3":
        live = nrows_all / steps_all   # keys per window step (each emits one row)
        pane = sum(per_batch) / len(per_batch)   # records per pane (a pane = one step's batch)
        alg = live * 26 * 2 + 2 * pane * 16 + live * 32
        unit = "one window step: R in + R' out (26 B per live key), entering + leaving pane (16 B per record), rows 32 B"
    else:
        kc = key.cpu().numpy()
        u = [len(np.unique(kc[s:e])) for s, e in bounds]
        alg = (24.0 * sum(per_batch) + 64.0 * sum(u)) / len(per_batch)
        unit = "one batch: 24 B per record + 2 x 32 B per distinct key (entry read and written)"
    roof = {"bound": "hbm", "kernel": dname, "alg_bytes_per_launch": alg, "alg_unit": unit, "peak": 8000.0,
            "unit": "GB/s", "avg_launch_ms": None, "achieved": None, "frac": None, "traffic": None,
            "kernel_stats": kernel_stats, "traffic_source": traffic}
    if kernel_stats and os.path.exists(kernel_stats):
        calls, avg = kernel_avg_ns(kernel_stats, dname)
        if avg:
            roof.update(avg_launch_ms=avg / 1e6, achieved=alg / avg, frac=alg / avg / 8000.0, launches_traced=calls)
    pmc_path = None
    if traffic and os.path.exists(traffic):
        tj = json.load(open(traffic)).get(cfg, {})
        if dname in tj:
            roof["traffic"] = tj[dname]["hbm_bytes_per_launch"]
        if kernel_stats and os.path.exists(kernel_stats) and tj:
            # measured bytes of the whole path: every traced kernel's PMC bytes per launch x its launches (the trace
            # covers the warm-up and timed steps of one drive), per step, over the timed run's time per step
            calls = kernel_calls(kernel_stats)
            # (generate_kernel: the synthetic source, run once before timing -- not part of the path)
            pb = sum(v["hbm_bytes_per_launch"] * calls.get(k, 0) for k, v in tj.items()
                     if not k.startswith("_") and k != "generate_kernel")
            per_step = pb / steps_all
            ms = elapsed / (len(bounds) - warm)
            pmc_path = {"bytes_per_step": per_step, "achieved": per_step / ms / 1e9, "unit": "GB/s",
                        "frac": per_step / ms / 1e9 / 8000.0, "measured_at": json.load(open(traffic)).get("_meta")}
    return {"metric": "records/sec per node, keyed window agg @1/2/4/8 GPU; % of HBM peak",
            "value": recs / elapsed, "unit": "records/s", "n_gpus": 1, "steps": len(bounds) - warm, "warmup": warm,
            "ms_per_step": elapsed / (len(bounds) - warm) * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int64", "data": "synthetic, resident in HBM before timing",
            "config": {"workload": workload, "records": n, "records_per_step": every, "pipelined_submit": pipe},
            "roofline": roof,
            "roofline_path": {"alg_bytes_lower_bound": path_bytes, "achieved": path_bytes / elapsed / 1e9,
                              "unit": "GB/s", "frac": path_bytes / elapsed / 1e9 / 8000.0},
            "roofline_pmc_path": pmc_path,
            "fired_rows": rows[0],
            "ms_per_step_profiled": None if prof_elapsed is None else prof_elapsed / (len(bounds) - warm) * 1e3,
            "kernels_ms": {k: {"launches": v[0], "total_ms": v[1]} for k, v in stats.items() if v[0]}}


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["c1", "c2", "c3", "c5"])
    ap.add_argument("--kernel-stats", default=None, help="rocprofv3 --stats CSV of this configuration ({cfg} is "
                                                          "replaced by the configuration name)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic_cfg.json"))
    a = ap.parse_args()
    for c in a.configs:
        ks = a.kernel_stats.replace("{cfg}", c) if a.kernel_stats else None
        print(json.dumps(run(c, ks, a.traffic)), flush=True)
