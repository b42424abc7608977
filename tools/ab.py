#!/usr/bin/env python3
"""Same-process A/B of engine environment knobs on one workload (experiments only).

usage: python tools/ab.py <workload> "<ENV=V ENV2=V>" "<...>" ...   (REPS=2, PASSES=2)
Each configuration gets a fresh Engine (knobs are read at engine creation), one
untimed pass, then PASSES timed passes (HIP events, fork to join); configurations
are interleaved REPS times so box drift hits all of them alike."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from shadow_amd.routes import SHDR_TIMING, Engine  # noqa: E402

wl, confs = sys.argv[1], sys.argv[2:] or [""]
reps, passes = int(os.environ.get("REPS", "2")), int(os.environ.get("PASSES", "2"))
nsrc = int(os.environ.get("NSRC", "0"))
if wl.startswith("gen:"):  # gen:<kind>:<n>:<hosts>  (experiments beyond the BASELINE configs)
    from shadow_amd.routes import Graph
    _, kind, n, nh = wl.split(":")
    g = Graph.generate(kind, int(n), 3, 1)
    hosts = np.sort(np.random.default_rng(1).permutation(g.V)[:int(nh)]).astype(np.int32)
else:
    g, hosts, _, _ = bench.make_workload(wl)
src = hosts[:nsrc] if nsrc else hosts
nparts = int(os.environ.get("PART", "0"))  # strong-scaling proxy: time every part of Engine.partition(hosts, PART)
parts = [src]
if nparts:
    part = Engine(g).partition(hosts, nparts)
    if os.environ.get("PART_RANDOM") == "1":  # same sizes, random membership (the control)
        part = np.random.default_rng(0).permutation(part)
    parts = [hosts[part == p] for p in range(min(nparts, int(os.environ.get("PARTS_MAX", nparts))))]
    src = parts[0]
dev = torch.device("cuda", 0)
S, T = max(len(x) for x in parts), len(hosts)
lat = torch.empty((S, T), dtype=torch.float64, device=dev)
rel = torch.empty((S, T), dtype=torch.float64, device=dev)
rmin = torch.empty((S,), dtype=torch.float64, device=dev)
res = {c: [] for c in confs}
base = dict(os.environ)
for r in range(reps):
    for c in confs:
        os.environ.clear()
        os.environ.update(base)
        for kv in c.split():
            k, v = kv.split("=", 1)
            os.environ[k] = v
        pc, pw = [], []
        for src in parts:
            eng = Engine(g)
            eng.compute_device(src, hosts, lat.data_ptr(), rel.data_ptr(), rmin.data_ptr(), None, flags=SHDR_TIMING)
            cold = eng.timing()["routes_pass"]
            lay0 = (eng.last_layout(), {k: round(v, 1) for k, v in eng.timing().items()}) if os.environ.get("VERBOSE_PARTS") else None
            ms = []
            for _ in range(passes):
                eng.compute_device(src, hosts, lat.data_ptr(), rel.data_ptr(), rmin.data_ptr(), None,
                                   flags=SHDR_TIMING)
                ms.append(eng.timing()["routes_pass"])
            pc.append(cold)
            pw.append(float(np.mean(ms)))
            if os.environ.get("VERBOSE_PARTS"):
                print(f"  part {len(pc) - 1}: rows {len(src)} cold {cold:.1f} warm {pw[-1]:.1f} layout cold {lay0} warm {eng.last_layout()}",
                      flush=True)
            del eng
        # a strong-scaling job waits for its slowest rank: the max over parts
        cold, ms = max(pc), [max(pw)]
        res[c].append((cold, ms))
        extra = f" (parts: mean {np.mean(pw):.1f} max {max(pw):.1f})" if len(parts) > 1 else ""
        print(f"rep {r} [{c}] cold {cold:.1f} warm {' '.join(f'{m:.1f}' for m in ms)}{extra}", flush=True)
print("== summary", wl, "S", S)
for c in confs:
    allw = [m for _, ms in res[c] for m in ms]
    print(f"[{c}] cold mean {np.mean([x for x, _ in res[c]]):.1f}  warm mean {np.mean(allw):.1f} min {np.min(allw):.1f}")
