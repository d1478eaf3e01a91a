# C5 session stream at reduced scale vs the numpy truth: max concurrent sessions per key.
import sys; sys.path.insert(0, "/root/repo"); sys.path.insert(0, ".")
import numpy as np
from bench_configs import session_stream
k, t, v = session_stream(100_000, 10_000_000, lag=5000)
print("n", len(k), "ts range", t.min(), t.max())
# per key sorted ts: count sessions and max gap structure
o = np.lexsort((t, k)); ks, ts = k[o], t[o]
newk = np.r_[True, ks[1:] != ks[:-1]]
gapbreak = np.r_[True, (ts[1:] - ts[:-1]) > 30_000]
sess = newk | gapbreak
print("sessions", sess.sum(), "per key", sess.sum() / 100_000)
# arrival-order check: how far behind the running max ts can a record be
run = np.maximum.accumulate(t)
print("max lag behind running max ts (ms)", int((run - t).max()))
