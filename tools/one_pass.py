#!/usr/bin/env python3
"""A few device-output table passes of one workload (profiling target; experiments only).
usage: python tools/one_pass.py <cfg4|cfg5> [passes=3]   (engine knobs from the environment)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from shadow_amd.routes import SHDR_TIMING, Engine  # noqa: E402

wl = sys.argv[1]
passes = int(sys.argv[2]) if len(sys.argv) > 2 else 3
g, hosts, _, _ = bench.make_workload(wl)
S = T = len(hosts)
dev = torch.device("cuda", 0)
lat = torch.empty((S, T), dtype=torch.float64, device=dev)
rel = torch.empty((S, T), dtype=torch.float64, device=dev)
rmin = torch.empty((S,), dtype=torch.float64, device=dev)
eng = Engine(g)
for i in range(passes):
    eng.compute_device(hosts, hosts, lat.data_ptr(), rel.data_ptr(), rmin.data_ptr(), None, flags=SHDR_TIMING)
    print(wl, i, {k: round(v, 1) for k, v in eng.timing().items() if not k.startswith("host_")}, flush=True)
