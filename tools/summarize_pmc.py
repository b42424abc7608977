#!/usr/bin/env python3
"""Print per-kernel PMC means (over dispatches) of a tools/gpu_pmc.sh session:
rows = counters, columns = runs (r<i>). usage: summarize_pmc.py gpurun_out/pmc"""
import collections
import csv
import os
import re
import sys

root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(list)))
for d in sorted(os.listdir(root)):
    m = re.match(r"r(\d+)_g(\d+)$", d)
    if not m:
        continue
    run = int(m.group(1))
    for dirpath, _, files in os.walk(os.path.join(root, d)):
        for f in files:
            if not f.endswith("counter_collection.csv"):
                continue
            per = collections.defaultdict(float)
            for r in csv.DictReader(open(os.path.join(dirpath, f))):
                k = re.sub(r"<.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
                           .split("(")[0]).strip()
                if "sssp" not in k and "k_routes" not in k:
                    continue
                disp = r.get("Dispatch_Id") or r.get("Correlation_Id")
                per[(k, r["Counter_Name"], disp)] += float(r["Counter_Value"])
            for (k, c, _), v in per.items():
                vals[k][c][run].append(v)
runs = sorted({r for k in vals for c in vals[k] for r in vals[k][c]})
for k in sorted(vals):
    print(f"== {k}")
    print("%-28s" % "counter" + "".join("%18s" % f"r{r}" for r in runs))
    for c in sorted(vals[k]):
        row = []
        for r in runs:
            xs = vals[k][c].get(r, [])
            row.append("%18.4g" % (sum(xs) / len(xs)) if xs else "%18s" % "-")
        print("%-28s" % c + "".join(row))
