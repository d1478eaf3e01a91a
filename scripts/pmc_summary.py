"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc_*/run_counter_collection.csv): per kernel, the
mean of each counter per dispatch (FETCH_SIZE/WRITE_SIZE in KB as rocprofv3 reports them)."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
vals = defaultdict(lambda: defaultdict(dict))   # kernel -> counter -> dispatch -> value
for f in sorted(glob.glob(f"{root}/pmc_*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][:48]
        c = r["Counter_Name"]
        d = vals[k][c]
        d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
# per kernel and counter: the mean over the dispatches of at least a tenth of the largest (a launch over an empty or
# tiny window -- the first fire of a run -- would otherwise halve a full fire's bytes)
acc = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(lambda: defaultdict(set))
for k in vals:
    for c, d in vals[k].items():
        top = max(d.values()) if d else 0.0
        keep = [i for i, x in d.items() if x >= 0.1 * top]
        acc[k][c] = sum(d[i] for i in keep)
        cnt[k][c] = set(keep)
for k in sorted(acc):
    print(k)
    for c in sorted(acc[k]):
        n = len(cnt[k][c])
        print(f"    {c:28s} {acc[k][c] / max(n, 1):16.1f}  (per dispatch, {n} dispatches of >= 1/10 of the largest)")


def traffic_json(out_path, root="gpurun_out"):
    """Writes {kernel: {"hbm_bytes_per_launch": B, ...}} from FETCH_SIZE/WRITE_SIZE passes, with the
    gfx950 correction of MI355X_MICROARCH.md (FETCH_SIZE counts half the bytes of wide coalesced
    reads: x2; WRITE_SIZE exact for 16-B streaming stores); both counters are in KB."""
    import json
    res = {}
    for k in acc:
        f = acc[k].get("FETCH_SIZE")
        w = acc[k].get("WRITE_SIZE")
        if f is None or w is None:
            continue
        nf, nw = len(cnt[k]["FETCH_SIZE"]), len(cnt[k]["WRITE_SIZE"])
        fb, wb = f / nf * 1024 * 2, w / nw * 1024
        name = k.split("::")[-1].split("<")[0]
        if name in res and res[name]["hbm_bytes_per_launch"] >= fb + wb:
            continue   # (another instance of the kernel, e.g. the fire's near-empty slow-list instance)
        res[name] = {"hbm_bytes_per_launch": fb + wb, "read_bytes": fb, "write_bytes": wb,
                     "launches_measured": nf, "note": "rocprofv3 FETCH_SIZE x2 (gfx950) + WRITE_SIZE, KB->B"}
    import datetime
    import os
    # the source tree the counters were taken on (TRAFFIC_HEAD: the git HEAD the gpurun command was sent from; the GPU
    # box has no .git), so a stale file shows in the bench line
    res["_meta"] = {"head": os.environ.get("TRAFFIC_HEAD", "unknown"),
                    "date": datetime.datetime.utcnow().strftime("%Y-%m-%d %H:%M UTC"),
                    "command": os.environ.get("TRAFFIC_CMD", "")}
    json.dump(res, open(out_path, "w"), indent=1)
    print("wrote", out_path)


if len(sys.argv) > 2:
    traffic_json(sys.argv[2], root)
