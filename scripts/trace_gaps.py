"""Per-step kernel timeline of a rocprofv3 kernel trace (the last K timed steps of bench.py): kernel durations,
the idle gaps between them, and totals per kernel.  Usage: trace_gaps.py run_kernel_trace.csv [steps]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void gwo::", "")
       .replace("gwo::", "")[:34]) for r in rows]
parts = [i for i, e in enumerate(ev) if "log_part" in e[2]]
first = parts[-steps]
# the timed region ends at the last gwo kernel after the last K1 (fire or pass 2)
last = max(i for i, e in enumerate(ev) if i >= first and ("log_" in e[2]))
tot = defaultdict(float)
cnt = defaultdict(int)
gap = 0.0
prev = None
for s, e, n in ev[first:last + 1]:
    if prev is not None:
        gap += max(0, s - prev) / 1e3
    tot[n] += (e - s) / 1e3
    cnt[n] += 1
    prev = e if prev is None else max(prev, e)
span = (ev[last][1] - ev[first][0]) / 1e3
print(f"span {span / steps:.1f} us/step, busy {sum(tot.values()) / steps:.1f} us/step, idle {gap / steps:.1f} us/step")
for n in sorted(tot, key=lambda k: -tot[k]):
    print(f"  {n:36s} {cnt[n]:4d} launches  {tot[n] / cnt[n]:9.1f} us avg  {tot[n] / steps:8.1f} us/step")
if "-v" in sys.argv:
    prev = None
    for s, e, n in ev[first:first + 12]:
        print(f"    {n:36s} dur {(e - s) / 1e3:8.1f} gap {(s - prev) / 1e3 if prev else 0:7.1f}")
        prev = e
