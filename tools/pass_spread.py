#!/usr/bin/env python3
"""Pass-to-pass spread of one table pass under engine knobs (same process, same box).

usage: python tools/pass_spread.py <workload> "<ENV=V ...>" "<...>"   (REPS=2, PASSES=8)
Each configuration gets a fresh Engine per repetition (knobs are read at engine
creation), one untimed pass, then PASSES timed passes; every pass's time (HIP
events, fork to join) is printed, with the tail launch's end (from the fork) when
the tail ran as a separate launch, and the layout. Configurations are interleaved
so box drift hits all alike. Outputs stay in HBM (bench.py's timed region)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from shadow_amd.routes import SHDR_TIMING, Engine, lib_kernel_sha  # noqa: E402

wl, confs = sys.argv[1], sys.argv[2:] or [""]
reps, passes = int(os.environ.get("REPS", "2")), int(os.environ.get("PASSES", "8"))
g, hosts, _, _ = bench.make_workload(wl)
dev = torch.device("cuda", 0)
S = T = len(hosts)
lat = torch.empty((S, T), dtype=torch.float64, device=dev)
rel = torch.empty((S, T), dtype=torch.float64, device=dev)
rmin = torch.empty((S,), dtype=torch.float64, device=dev)
print(f"# {wl}: S = T = {S}, lib_sha {lib_kernel_sha()}, {reps} reps x {passes} passes per config", flush=True)
res = {c: [] for c in confs}
tails = {c: [] for c in confs}
base = dict(os.environ)
for r in range(reps):
    for c in confs:
        os.environ.clear()
        os.environ.update(base)
        for kv in c.split():
            k, v = kv.split("=", 1)
            os.environ[k] = v
        eng = Engine(g)
        eng.compute_device(hosts, hosts, lat.data_ptr(), rel.data_ptr(), rmin.data_ptr(), None, flags=SHDR_TIMING)
        ms, tl = [], []
        for _ in range(passes):
            eng.compute_device(hosts, hosts, lat.data_ptr(), rel.data_ptr(), rmin.data_ptr(), None, flags=SHDR_TIMING)
            t = eng.timing()
            ms.append(t["routes_pass"])
            if "k_routes_sssp_tail" in t:
                tl.append(t["k_routes_sssp_tail"])
        res[c] += ms
        tails[c] += tl
        lay = eng.last_layout()
        print(f"rep {r} [{c}] tail_mode {lay['tail_mode']} rows_main {lay['rows_main']} passes "
              + " ".join(f"{m:.1f}" for m in ms) + (("  tail ends " + " ".join(f"{x:.1f}" for x in tl)) if tl else ""),
              flush=True)
        del eng
print("== summary", wl)
for c in confs:
    a = np.array(res[c])
    line = f"[{c}] passes {len(a)} mean {a.mean():.1f} min {a.min():.1f} max {a.max():.1f} (max-min)/mean {np.ptp(a) / a.mean():.3f}"
    if tails[c]:
        t = np.array(tails[c])
        line += f"; tail end mean {t.mean():.1f} min {t.min():.1f} max {t.max():.1f}"
    print(line, flush=True)
