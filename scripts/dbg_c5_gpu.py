import sys; sys.path.insert(0, "/root/repo"); sys.path.insert(0, ".")
import numpy as np
import flink_amd as F
from bench_configs import session_stream
nk = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000
k, t, v = session_stream(nk, nk * 100, lag=5000)
every = len(k) // 100
op = F.GpuWindowOperator(F.EventTimeSessionWindows.withGap(30_000), F.SumAggregate())
run = -(1 << 63)
for i, s in enumerate(range(0, len(k), every)):
    e = min(s + every, len(k))
    run = max(run, int(t[s:e].max()))
    try:
        op.process_batch(k[s:e], t[s:e], v[s:e]); op.process_watermark(run - 5001)
    except Exception as ex:
        print("batch", i, "failed:", ex); break
    if i % 10 == 0: print("batch", i, "wm", run - 5001, "live sessions", op.state_size, "rows", len(op.output))
