#!/usr/bin/env python3
"""Vertex numbering experiment: kernel time under relabelings of the same graph
(original, random, BFS from the hub, degree-descending, RCM, distance from the hub).
Run with SHDR_RELABEL=0 so the engine keeps the given numbering.
usage: exp_perm.py [cfg4|cfg5] [comma-separated orders]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
from scipy.sparse import csgraph  # noqa: E402

import bench  # noqa: E402
from shadow_amd.routes import SHDR_TIMING, Engine, Graph  # noqa: E402

g, hosts, _, _ = bench.make_workload(sys.argv[1] if len(sys.argv) > 1 else "cfg4")
ef, et, lat, lo, vl = g.export()
V = g.V
m = ef != et
A = sp.coo_matrix((np.ones(m.sum()), (ef[m], et[m])), shape=(V, V)).tocsr()
A = A + A.T
deg = np.diff(A.indptr)
hub = int(np.argmax(deg))
orders = {
    "original": np.arange(V),
    "random": np.random.default_rng(0).permutation(V),
    "bfs": csgraph.breadth_first_order(A, hub, directed=False, return_predecessors=False),
    "degree": np.argsort(-deg, kind="stable"),
    "rcm": csgraph.reverse_cuthill_mckee(A.tocsr(), symmetric_mode=True)[::-1].copy(),
}
W = sp.coo_matrix((lat[m], (ef[m], et[m])), shape=(V, V)).tocsr()
orders["hubdist"] = np.argsort(csgraph.dijkstra(W, directed=False, indices=hub), kind="stable")
if len(sys.argv) > 2:
    orders = {k: orders[k] for k in sys.argv[2].split(",")}
for name, order in orders.items():
    newid = np.empty(V, np.int64)
    newid[order] = np.arange(V)
    g2 = Graph.from_edges(V, newid[ef], newid[et], lat, lo, vl[order])
    eng = Engine(g2)
    h2 = newid[hosts].astype(np.int32)
    eng.compute(h2[:256], h2)
    ms = []
    for _ in range(2):
        eng.compute(h2, h2, flags=SHDR_TIMING)
        ms.append(eng.timing().get('routes_pass', sum(eng.timing().values())))
    print(f"{name:9s} kernel_ms={min(ms):.1f}", flush=True)
