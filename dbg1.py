import sys, json, ctypes as C
sys.path.insert(0, '.')
import numpy as np
import flink_amd as F
from flink_amd import _native as N
from oracle import gen as G
g = json.load(open('tests/golden/reference_vectors.json'))
s = next(x for x in g['operator_streams'] if x['name']=="tumbling_3s")
for pre in ("1", "0"):
    import os; os.environ["GWO_PREAGG"] = pre
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(3000), F.SumAggregate())
    lib = N.lib(); h = op.handle
    for ev in s['events']:
        if ev[0]=='e': op.process_element(ev[1], ev[2], ev[3])
        else:
            op.flush()
            print("pre", pre, "wm", ev[1], "state", op.state_size(), flush=True)
            n = C.c_int64()
            st = lib.gwo_advance_watermark(h, ev[1]); lib.gwo_output_count(h, C.byref(n))
            print("  adv st", st, "out_rows", n.value, lib.gwo_last_error(h), flush=True)
            op._collect()
    print("got", sorted(op.output), flush=True)
import torch
spec = G.GenSpec(seed=7, first_index=123, total_records=10**6, num_keys=5000, span_ms=60000, disorder_ms=1000, value_range=1000)
n=8
k = torch.empty(n, dtype=torch.int64, device="cuda"); t = torch.empty_like(k); v = torch.empty_like(k)
gs = N.GwoGenSpec(spec.seed, spec.first_index, spec.total_records, spec.num_keys, spec.span_ms, spec.disorder_ms, spec.t0, spec.value_range, 0, 0)
print("gen st", N.lib().gwo_generate(C.byref(gs), n, k.data_ptr(), t.data_ptr(), v.data_ptr(), None, 0))
wk, wt, wv = G.generate(spec, n)
print("k", k.cpu().tolist(), wk.tolist()); print("t", t.cpu().tolist(), wt.tolist()); print("v", v.cpu().tolist(), wv.tolist(), flush=True)
