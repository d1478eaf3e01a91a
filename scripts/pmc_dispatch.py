"""Per-dispatch table of rocprofv3 --pmc passes written by scripts/gpu_pmc_py.sh (gpurun_out/<tag>_<i>/):
one line per dispatch of each kernel with every counter collected for it, plus per-kernel means.  FETCH_SIZE and
WRITE_SIZE are in KB as rocprofv3 reports them; HBM bytes = FETCH_SIZE x 2 (the gfx950 correction of
MI355X_MICROARCH.md for wide coalesced reads) + WRITE_SIZE.  Passes are separate runs of the same deterministic
program, so dispatch i of a kernel is the same launch in every pass.

usage: python scripts/pmc_dispatch.py gpurun_out/<tag> [kernel-substring] [--all]"""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
only = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else None
show_all = "--all" in sys.argv
per = defaultdict(lambda: defaultdict(dict))   # kernel -> dispatch ordinal -> counter -> value
for f in sorted(glob.glob(f"{root}_*/run_counter_collection.csv")):
    seen = defaultdict(list)
    rows = list(csv.DictReader(open(f)))
    for r in rows:
        k = r["Kernel_Name"].split("(")[0]
        if only and only not in k:
            continue
        d = int(r["Dispatch_Id"])
        if d not in seen[k]:
            seen[k].append(d)
    for r in rows:
        k = r["Kernel_Name"].split("(")[0]
        if only and only not in k:
            continue
        i = seen[k].index(int(r["Dispatch_Id"]))
        per[k][i][r["Counter_Name"]] = per[k][i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k, ds in per.items():
    print(k)
    counters = sorted({c for d in ds.values() for c in d})
    means = {c: sum(d.get(c, 0) for d in ds.values()) / len(ds) for c in counters}
    print("  mean over", len(ds), "dispatches:", ", ".join(f"{c}={means[c]:.1f}" for c in counters))
    if "FETCH_SIZE" in means and "WRITE_SIZE" in means:
        print(f"  mean HBM bytes/dispatch: {(2 * means['FETCH_SIZE'] + means['WRITE_SIZE']) * 1024 / 1e6:.1f} MB")
    if show_all:
        for i in sorted(ds):
            d = ds[i]
            hbm = ""
            if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
                hbm = f"  HBM {(2 * d['FETCH_SIZE'] + d['WRITE_SIZE']) * 1024 / 1e6:.1f} MB"
            print(f"  #{i}: " + ", ".join(f"{c}={d[c]:.0f}" for c in sorted(d)) + hbm)
