"""Per-step GPU timeline from a rocprofv3 kernel trace: each op's duration and the idle gap before it."""
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/trace"
rows = sorted(csv.DictReader(open(f"{d}/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "log_part" in r["Kernel_Name"]]
prev = None
busy = idle = 0.0
for r in rows[idx[-12]:idx[-1] + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f"{r['Kernel_Name'][:48]:48s} dur={(e - s) / 1e3:8.1f}us gap_before={gap:7.1f}us")
    busy += (e - s) / 1e3
    idle += max(gap, 0)
    prev = e
print(f"busy {busy:.1f} us, idle {idle:.1f} us over 11 steps")
