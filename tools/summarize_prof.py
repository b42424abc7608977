#!/usr/bin/env python3
"""Summarise a tools/profile.sh output dir into profiles/pmc_<workload>.json
(+ a copy of the rocprofv3 --kernel-trace --stats CSV as
profiles/<tag>_kernel_stats.csv).

The routes.hip sha recorded by tools/profile.sh on the box is copied into the
summary (bench.load_pmc_traffic ignores a summary of another kernel), and so is
the bench line of the profiled run itself (same session as the counters).

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are KiB
per dispatch; on gfx950 FETCH_SIZE tallies 128-B requests at 64 B, so read
bytes = 2 x FETCH_SIZE. The calibration pass (tools/ubench under --pmc
FETCH_SIZE) checks that factor on this access pattern: a 128-B random row
gather and a coalesced stream with known byte counts.

usage: tools/summarize_prof.py <prof dir> <tag> <workload> <sources per launch>
"""
import collections
import csv
import json
import os
import re
import shutil
import sys

src, tag, workload, per = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kname(raw):
    k = raw.replace("(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"<.*", "", k.split("(")[0]).strip()


def counters(sub):
    """-> {kernel: {counter: [per-dispatch values]}}"""
    out = collections.defaultdict(lambda: collections.defaultdict(dict))
    d = os.path.join(src, sub)
    for dirpath, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                for r in csv.DictReader(open(os.path.join(dirpath, f))):
                    k = kname(r["Kernel_Name"])
                    disp = r.get("Dispatch_Id") or r.get("Correlation_Id")
                    out[k][r["Counter_Name"]][disp] = out[k][r["Counter_Name"]].get(disp, 0.0) + float(r["Counter_Value"])
    return {k: {c: list(v.values()) for c, v in cs.items()} for k, cs in out.items()}


durations = {}
for dirpath, _, files in os.walk(os.path.join(src, "ktrace")):
    for f in files:
        if f.endswith("kernel_stats.csv"):
            p = os.path.join(dirpath, f)
            for r in csv.DictReader(open(p)):
                durations[kname(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
            shutil.copyfile(p, os.path.join(root, "profiles", f"{tag}_kernel_stats.csv"))
sha_file = os.path.join(src, "kernel_sha")
kernel_sha = open(sha_file).read().strip() if os.path.exists(sha_file) else None
bench_line = None
bl = os.path.join(src, "bench_line.json")
if os.path.exists(bl) and os.path.getsize(bl):
    bench_line = json.loads(open(bl).read())
res = {"workload": workload, "sources_per_launch": per, "source": src, "kernel_sha": kernel_sha,
       "bench_line_same_session": bench_line,
       "method": "rocprofv3 separate --pmc passes: FETCH_SIZE, WRITE_SIZE, TCC_HIT_sum+TCC_MISS_sum; "
                 "bytes = 2*1024*FETCH_SIZE + 1024*WRITE_SIZE per dispatch (gfx950 FETCH_SIZE correction)",
       "kernels": {}}
agg = collections.defaultdict(dict)
for sub in ("fetch", "write", "tcc"):
    for k, cs in counters(sub).items():
        for c, vals in cs.items():
            agg[k][c] = sum(vals) / max(len(vals), 1)
for k, c in agg.items():
    e = dict(c)
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        e["hbm_read_bytes_per_launch"] = 2.0 * 1024.0 * c["FETCH_SIZE"]
        e["hbm_write_bytes_per_launch"] = 1024.0 * c["WRITE_SIZE"]
        e["hbm_bytes_per_launch"] = e["hbm_read_bytes_per_launch"] + e["hbm_write_bytes_per_launch"]
    if k in durations:
        e.update(durations[k])
        if "hbm_bytes_per_launch" in e:
            e["hbm_GBps"] = e["hbm_bytes_per_launch"] / durations[k]["avg_ns"]
    if "TCC_HIT_sum" in c:
        e["l2_hit_rate"] = c["TCC_HIT_sum"] / max(c["TCC_HIT_sum"] + c["TCC_MISS_sum"], 1)
    res["kernels"][k] = e
cal = counters("calib")
if cal:
    # tools/ubench 4096: stream = 4 GiB read once; gather<16> = 4096*256/16*256 rows of 128 B
    known = {"k_stream": 4096 * 2**20, "k_gather": None}
    res["calibration"] = {k: {"FETCH_SIZE_KiB_per_dispatch": cs.get("FETCH_SIZE", [])} for k, cs in cal.items()}
    if "k_stream" in cal and cal["k_stream"].get("FETCH_SIZE"):
        f = cal["k_stream"]["FETCH_SIZE"][-1] * 1024.0
        res["calibration"]["stream_known_bytes"] = known["k_stream"]
        res["calibration"]["stream_fetch_bytes"] = f
        res["calibration"]["stream_ratio_known_over_fetch"] = known["k_stream"] / f
    if "k_gather" in cal:
        rows = 4096 * 256 // 16 * 256
        vals = cal["k_gather"].get("FETCH_SIZE", [])
        # dispatches in order: rows of 8,16,...,512 B then 128-B rows in 2/32/192 MiB
        res["calibration"]["gather_rows_per_dispatch_128B"] = rows
        res["calibration"]["gather_fetch_bytes_per_dispatch"] = [v * 1024.0 for v in vals]
json.dump(res, open(os.path.join(root, "profiles", f"pmc_{workload}.json"), "w"), indent=1)
print(json.dumps(res["kernels"], indent=1))
print(json.dumps(res.get("calibration", {}), indent=1)[:2000])
