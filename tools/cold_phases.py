#!/usr/bin/env python3
"""Cold-path phase split on cfg5 (experiments only): engine start-up phases
(SHDR_VERBOSE=1 prints csr / relabel / upload / blocks+items on stderr) and the
first compute's host phases (landmarks, grouping, launch, pass), into device
buffers so no D2H is counted."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("SHDR_VERBOSE", "1")
import numpy as np  # noqa: E402
import torch  # noqa: E402

from shadow_amd.routes import Engine, Graph  # noqa: E402

g = Graph.generate("chunglu", 1_000_000, 3, 1)
hosts = np.sort(np.random.default_rng(1).choice(g.V, 50_000, replace=False)).astype(np.int32)
torch.cuda.init()
t0 = time.perf_counter()
eng = Engine(g)
t1 = time.perf_counter()
S = T = len(hosts)
lat = torch.empty((S, T), dtype=torch.float64, device="cuda")
rel = torch.empty_like(lat)
rmin = torch.empty((S,), dtype=torch.float64, device="cuda")
t2 = time.perf_counter()
eng.compute_device(hosts, hosts, lat.data_ptr(), rel.data_ptr(), rmin.data_ptr(), None, flags=4)
torch.cuda.synchronize()
t3 = time.perf_counter()
print(f"engine_create {1e3 * (t1 - t0):.1f} ms, first compute {1e3 * (t3 - t2):.1f} ms", flush=True)
print({k: round(v, 1) for k, v in eng.timing().items()}, flush=True)
