import sys; sys.path.insert(0, "/root/repo"); sys.path.insert(0, ".")
import numpy as np
import flink_amd as F
from oracle import gen as G, vectorized as V
LONG_MAX = (1 << 63) - 1
spec = G.GenSpec(seed=42, total_records=1_000_000, num_keys=200_000, span_ms=60000, disorder_ms=50, value_range=1000)
k, t, v = G.generate(spec, 1_000_000)
b = G.punctuated_watermarks(t, 10_000, 100)
agg = F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.MaxAggregate())
op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(60000), agg, state_layout="log")
prev = 0
for end, wm in b:
    op.process_batch(k[prev:end], t[prev:end], v[prev:end]); op.process_watermark(wm); prev = end
op.end_input()
(wk, ws, we, res), late = V.tumbling_lateness0(k, t, v, b + [(b[-1][0], LONG_MAX)], 60000, 0, [1, 2, 3])
want = {(a, s): tuple(r) for a, s, r in zip(wk.tolist(), ws.tolist(), zip(*[x.tolist() for x in res]))}
got = {}
dup = 0
for a, s, e, r in op.output:
    if (a, s) in got: dup += 1
    got[(a, s)] = tuple(r)
missing = [x for x in want if x not in got]; extra = [x for x in got if x not in want]
diff = [x for x in want if x in got and got[x] != want[x]]
print("rows got", len(op.output), "want", len(want), "dup", dup, "missing", len(missing), "extra", len(extra), "diff", len(diff))
for x in diff[:5]: print("diff", x, got[x], want[x])
for x in missing[:3]: print("missing", x, want[x])
