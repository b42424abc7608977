#!/usr/bin/env python3
"""Arena placement experiment (experiments only): one workload, a fresh engine per
trial (SHDR_VERBOSE prints each arena address), cold + PASSES timed passes.
usage: python tools/alloc_var.py <workload> <trials> ["ENV=V ..." per block]..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from shadow_amd.routes import SHDR_TIMING, Engine  # noqa: E402

wl, trials = sys.argv[1], int(sys.argv[2])
g, hosts, _, _ = bench.make_workload(wl)
S = T = len(hosts)
dev = torch.device("cuda", 0)
lat = torch.empty((S, T), dtype=torch.float64, device=dev)
rel = torch.empty((S, T), dtype=torch.float64, device=dev)
rmin = torch.empty((S,), dtype=torch.float64, device=dev)
os.environ["SHDR_VERBOSE"] = "1"
base = dict(os.environ)
for block in sys.argv[3:] or [""]:
    for t in range(trials):
        os.environ.clear()
        os.environ.update(base)
        for kv in block.split():
            k, v = kv.split("=", 1)
            os.environ[k] = v
        eng = Engine(g)
        ms = []
        for p in range(1 + int(os.environ.get("PASSES", "2"))):
            eng.compute_device(hosts, hosts, lat.data_ptr(), rel.data_ptr(), rmin.data_ptr(), None, flags=SHDR_TIMING)
            ms.append(eng.timing()["routes_pass"])
        print(f"[{block}] trial {t}: " + " ".join(f"{m:.1f}" for m in ms), flush=True)
        del eng
