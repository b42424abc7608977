#!/usr/bin/env python3
"""Summarise a tools/profile.sh output dir into profiles/<name>.json (+ copy the
rocprofv3 --kernel-trace --stats CSV). HBM bytes follow MI355X_MICROARCH.md
§HBM: FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the
bytes of wide coalesced reads, so the corrected read bytes are 2 x FETCH_SIZE."""
import collections
import csv
import json
import os
import shutil
import sys

src, name = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = {"source": src}
per_kernel = collections.defaultdict(lambda: collections.defaultdict(float))
launches = collections.Counter()
for sub in ("fetch", "write", "tcc", "sq"):
    p = os.path.join(src, sub, "run_counter_collection.csv")
    if not os.path.exists(p):
        continue
    seen = set()
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        per_kernel[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if sub == "fetch" and (r["Dispatch_Id"], k) not in seen:
            seen.add((r["Dispatch_Id"], k))
            launches[k] += 1
stats = os.path.join(src, "ktrace", "run_kernel_stats.csv")
durations = {}
if os.path.exists(stats):
    for r in csv.DictReader(open(stats)):
        k = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        durations[k] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "total_ns": float(r["TotalDurationNs"])}
    shutil.copyfile(stats, os.path.join(root, "profiles", f"{name}_kernel_stats.csv"))
for k, c in per_kernel.items():
    n = max(launches.get(k, 1), 1)
    e = {kk: v / n for kk, v in c.items()}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        e["hbm_read_bytes_per_launch"] = 2.0 * 1024.0 * c["FETCH_SIZE"] / n
        e["hbm_write_bytes_per_launch"] = 1024.0 * c["WRITE_SIZE"] / n
        e["hbm_bytes_per_launch"] = e["hbm_read_bytes_per_launch"] + e["hbm_write_bytes_per_launch"]
    if k in durations:
        e["avg_ns"] = durations[k]["avg_ns"]
        if "hbm_bytes_per_launch" in e:
            e["hbm_GBps"] = e["hbm_bytes_per_launch"] / durations[k]["avg_ns"]
    if "TCC_HIT_sum" in c:
        e["l2_hit_rate"] = c["TCC_HIT_sum"] / max(c["TCC_HIT_sum"] + c["TCC_MISS_sum"], 1)
    out[k] = e
json.dump(out, open(os.path.join(root, "profiles", f"{name}.json"), "w"), indent=1)
print(json.dumps({k: {kk: round(v, 3) if isinstance(v, float) else v for kk, v in e.items()} for k, e in out.items() if k != "source"}, indent=1))
