"""Multi-GPU path on the CPU: key-group sharding over world_size 2 with torch.distributed
gloo, the same contract the RCCL path implements on the GPU (gwo_comm.cpp):

  * rank g owns computeKeyGroupRangeForOperatorIndex(maxP, G, g) (KeyGroupRangeAssignment.java:88-101);
  * every record is routed to computeOperatorIndexForKeyGroup(assignToKeyGroup(key)) (:48-73,118-119) by
    one all-to-all per batch (KeyGroupStreamPartitioner.selectChannel, KeyGroupStreamPartitioner.java:51-58);
  * the watermark is the min over ranks (StatusWatermarkValve.java:163-181);
  * the union of the ranks' window outputs equals the single-operator oracle output.

The per-rank window aggregation here is the oracle (test infrastructure); the GPU test of the same
exchange through libgwo.so's RCCL path is tests/test_gpu_windows.py::test_comm_*.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from flink_amd.keygroups import compute_key_group_range_for_operator_index
from oracle import flink_oracle as O
from oracle import gen as G
from oracle import vectorized as V

WORLD = 2
MAXP = 128


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _stream():
    spec = G.GenSpec(seed=7, total_records=120_000, num_keys=5_000, span_ms=30_000, disorder_ms=800, value_range=1000)
    k, t, v = G.generate(spec, spec.total_records)
    return k, t, v


def _worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        k, t, v = _stream()
        rng = compute_key_group_range_for_operator_index(MAXP, WORLD, rank)
        # this rank is the source of records [rank::WORLD] (its input split), in arrival order
        src = np.arange(rank, len(k), WORLD)
        batches = 12
        per = (len(src) + batches - 1) // batches
        rk, rt, rv = [], [], []
        wm_seen = []
        for b in range(batches):
            idx = src[b * per:(b + 1) * per]
            _, dest = V.key_groups(k[idx], MAXP, WORLD)
            order = np.argsort(dest, kind="stable")            # grouped by destination, arrival order kept
            send = np.stack([k[idx][order], t[idx][order], v[idx][order]], 1).astype(np.int64)
            counts = torch.tensor(np.bincount(dest, minlength=WORLD), dtype=torch.int64)
            rcounts = torch.empty(WORLD, dtype=torch.int64)
            dist.all_to_all_single(rcounts, counts)
            out = torch.empty((int(rcounts.sum()), 3), dtype=torch.int64)
            dist.all_to_all_single(out, torch.from_numpy(send), rcounts.tolist(), counts.tolist())
            got = out.numpy()
            kg, _ = V.key_groups(got[:, 0], MAXP, WORLD)
            assert ((kg >= rng.start_key_group) & (kg <= rng.end_key_group)).all(), "record routed to a non-owner"
            rk.append(got[:, 0]), rt.append(got[:, 1]), rv.append(got[:, 2])
            # watermark after the batch: each source's max ts - lag, combined by min over ranks
            local_wm = torch.tensor([int(t[idx].max()) - 5_000 - 1], dtype=torch.int64)
            dist.all_reduce(local_wm, op=dist.ReduceOp.MIN)
            wm_seen.append(int(local_wm))
        rk, rt, rv = np.concatenate(rk), np.concatenate(rt), np.concatenate(rv)
        # lag 5 s > disorder: no record is late, so the output set does not depend on watermark timing
        (wk, ws, we, res), late = V.tumbling_lateness0(rk, rt, rv, [(len(rk), O.LONG_MAX)], 5000, 0, [1, 2, 3])
        assert late == 0
        rows = list(zip(wk.tolist(), ws.tolist(), we.tolist(), *[x.tolist() for x in res]))
        gathered = [None] * WORLD
        dist.all_gather_object(gathered, rows)
        if rank == 0:
            q.put((gathered, wm_seen))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_keygroup_sharded_window_agg_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    gathered, wms = q.get(timeout=150)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    k, t, v = _stream()
    (wk, ws, we, res), _ = V.tumbling_lateness0(k, t, v, [(len(k), O.LONG_MAX)], 5000, 0, [1, 2, 3])
    want = sorted(zip(wk.tolist(), ws.tolist(), we.tolist(), *[x.tolist() for x in res]))
    union = sorted(r for part in gathered for r in part)
    assert union == want
    keys0 = {r[0] for r in gathered[0]}
    keys1 = {r[0] for r in gathered[1]}
    assert not keys0 & keys1, "a key was aggregated on two ranks"
    assert wms == sorted(wms), "min-over-ranks watermark must be monotone here"


def test_numpy_key_groups_match_loop_oracle():
    rng = np.random.default_rng(3)
    keys = np.concatenate([rng.integers(-(1 << 63), (1 << 63) - 1, 2000, dtype=np.int64),
                           np.array([0, 1, -1, O.LONG_MIN, O.LONG_MAX], np.int64)])
    for maxp, par in ((128, 2), (32768, 8), (32768, 3), (1, 1)):
        kg, op = V.key_groups(keys, maxp, par)
        for x, g, o in zip(keys.tolist(), kg.tolist(), op.tolist()):
            h = O.long_hash_code(x)
            assert g == O.assign_to_key_group(h, maxp)
            assert o == O.compute_operator_index_for_key_group(maxp, par, g)


def test_key_group_ranges_partition_all_groups():
    for maxp in (128, 32768):
        for par in (1, 2, 4, 8):
            seen = []
            for i in range(par):
                r = compute_key_group_range_for_operator_index(maxp, par, i)
                seen.extend(range(r.start_key_group, r.end_key_group + 1))
                kg = np.arange(r.start_key_group, r.end_key_group + 1)
                assert ((kg * par) // maxp == i).all()   # routing and ownership agree
            assert seen == list(range(maxp))
