#!/usr/bin/env python3
"""Tail experiment: time k_routes_sssp on sub-ranges of the cfg4 sources."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from shadow_amd.routes import SHDR_TIMING, Engine  # noqa: E402

g, hosts, _, _ = bench.make_workload("cfg4")
eng = Engine(g)
for var, lo, hi in [(4, 0, 10000), (4, 0, 8192), (4, 8192, 10000), (6, 8192, 10000), (0, 8192, 10000),
                    (4, 0, 4096), (4, 0, 1250), (6, 0, 1250), (0, 0, 1250), (1, 0, 1250), (4, 0, 16), (6, 0, 8)]:
    eng.set_variant(var)
    src = hosts[lo:hi]
    eng.compute(src, hosts)
    ms = []
    for _ in range(2):
        eng.compute(src, hosts, flags=SHDR_TIMING)
        ms.append(eng.timing().get('routes_pass', sum(eng.timing().values())))
    print(f"variant {var} sources [{lo},{hi}) n={hi-lo} kernel {min(ms):.1f} ms", flush=True)
