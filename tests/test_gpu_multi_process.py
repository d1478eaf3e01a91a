"""World-2 keyBy shuffle with libgwo.so in two processes, on one GPU.

Each rank is one operator subtask: a GpuWindowOperator owning computeKeyGroupRangeForOperatorIndex(maxP, 2, rank)
(KeyGroupRangeAssignment.java:88-101).  Its input split is routed on the GPU by gwo_partition_by_operator
(KeyGroupStreamPartitioner.selectChannel, KeyGroupStreamPartitioner.java:51-58; gwo.h's route step for hosts with
their own transport), exchanged with torch.distributed gloo all-to-all, and submitted to the rank's handle; the
watermark after each batch is the min over ranks (StatusWatermarkValve.java:163-181).  The splits are unequal (70/30),
so every batch carries different counts per peer, and the lag is below the disorder, so records arrive late.

Per rank, the rows and the late-record count equal the oracle run over exactly the records that rank received, in
its batches, with the agreed watermarks; the ranks' keys are disjoint.  (tests/test_multi.py is the CPU contract test
of the same exchange; the RCCL path of gwo_comm is covered by tests/test_gpu_windows.py::test_comm_*.)
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WORLD = 2
MAXP = 128
LAG = 300            # < the stream's disorder (3 s): late records exist


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _stream():
    from oracle import gen as G
    spec = G.GenSpec(seed=11, total_records=200_000, num_keys=6_000, span_ms=40_000, disorder_ms=3000,
                     value_range=1000)
    return G.generate(spec, spec.total_records)


def _worker(rank, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        import torch
        import flink_amd as F
        from flink_amd import _native as N
        from flink_amd.keygroups import compute_key_group_range_for_operator_index
        from oracle import flink_oracle as O
        from oracle import vectorized as V

        k, t, v = _stream()
        rng = compute_key_group_range_for_operator_index(MAXP, WORLD, rank)
        mine = (np.arange(len(k)) % 10 < 7) == (rank == 0)   # this rank's source split, in arrival order
        src = np.flatnonzero(mine)
        op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(5000),
                                 F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.MaxAggregate()),
                                 max_parallelism=MAXP, key_group_range=(rng.start_key_group, rng.end_key_group))
        lib = N.lib()
        batches = 40
        per = (len(src) + batches - 1) // batches
        rk, rt, rv, marks = [], [], [], []
        received = 0
        for b in range(batches):
            idx = src[b * per:(b + 1) * per]
            bk, bt, bv = (np.ascontiguousarray(x[idx]) for x in (k, t, v))
            n = len(idx)
            cap = max(n, 1)
            out = np.zeros(WORLD * cap * 3, np.int64)
            counts = np.zeros(WORLD, np.int64)
            ptr = lambda a: a.ctypes.data_as(C.c_void_p)
            N.check(lib.gwo_partition_by_operator(ptr(bk), ptr(bt), ptr(bv), n, N.KEY_LONG, MAXP, WORLD, ptr(out),
                                                  cap, ptr(counts), 0))
            assert int(counts.sum()) == n and (counts <= cap).all()
            send = np.concatenate([out[p * cap * 3:p * cap * 3 + int(counts[p]) * 3] for p in range(WORLD)])
            rcounts = torch.empty(WORLD, dtype=torch.int64)
            dist.all_to_all_single(rcounts, torch.from_numpy(counts.copy()))
            got = torch.empty(int(rcounts.sum()) * 3, dtype=torch.int64)
            dist.all_to_all_single(got, torch.from_numpy(send), [int(c) * 3 for c in rcounts.tolist()],
                                   [int(c) * 3 for c in counts.tolist()])
            got = got.numpy().reshape(-1, 3)
            kg, _ = V.key_groups(got[:, 0], MAXP, WORLD)
            assert ((kg >= rng.start_key_group) & (kg <= rng.end_key_group)).all(), "record routed to a non-owner"
            op.process_batch(got[:, 0], got[:, 1], got[:, 2])
            rk.append(got[:, 0]), rt.append(got[:, 1]), rv.append(got[:, 2])
            received += len(got)
            local = torch.tensor([int(bt.max()) - LAG - 1 if n else O.LONG_MIN], dtype=torch.int64)
            dist.all_reduce(local, op=dist.ReduceOp.MIN)
            wm = int(local)
            op.process_watermark(wm)
            marks.append((received, wm))
        op.end_input()
        rows = sorted((a, s, e, *r) for a, s, e, r in op.output)
        late = op.num_late_records_dropped
        op.close()
        RK, RT, RV = (np.concatenate(x) for x in (rk, rt, rv))
        (wk, ws, we, res), olate = V.tumbling_lateness0(RK, RT, RV, marks + [(received, O.LONG_MAX)], 5000, 0,
                                                        [1, 2, 3])
        want = sorted(zip(wk.tolist(), ws.tolist(), we.tolist(), *[x.tolist() for x in res]))
        gathered = [None] * WORLD
        dist.all_gather_object(gathered, (rows == want, len(rows), late, olate, sorted({r[0] for r in rows}),
                                          received, len(src)))
        if rank == 0:
            q.put(gathered)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_two_processes_route_exchange_and_aggregate_like_the_oracle():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=200)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    k, _, _ = _stream()
    assert sum(g[5] for g in gathered) == len(k)                       # every record reached exactly one owner
    assert gathered[0][6] > 2 * gathered[1][6]                        # unequal sources: rank 0 sends 70 %
    for equal, nrows, late, olate, _, _, _ in gathered:
        assert equal and nrows > 1000
        assert late == olate
    assert sum(g[2] for g in gathered) > 0, "the stream should carry late records"
    assert not set(gathered[0][4]) & set(gathered[1][4]), "a key was aggregated on two ranks"
