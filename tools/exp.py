#!/usr/bin/env python3
"""Kernel-time sweep over engine variants / delta on a workload (experiments only).
usage: python tools/exp.py <workload> <variant,...> [delta,...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from shadow_amd.routes import SHDR_TIMING, Engine  # noqa: E402
import bench  # noqa: E402

wl = sys.argv[1]
variants = [int(x) for x in sys.argv[2].split(",")]
deltas = [float(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0.0]
nsrc = int(os.environ.get("EXP_NSRC", "0"))
g, hosts, _pool, desc = bench.make_workload(wl)
src = hosts[:nsrc] if nsrc else hosts
order = os.environ.get("EXP_ORDER", "")
if order:
    import scipy.sparse as sp
    from scipy.sparse import csgraph
    ef, et, lat, _, _ = g.export()
    m = ef != et
    A = sp.coo_matrix((lat[m], (ef[m], et[m])), shape=(g.V, g.V)).tocsr()
    A = A + A.T
    deg = np.diff(A.indptr)
    hub = int(np.argmax(deg))
    if order == "bfs":
        bo = csgraph.breadth_first_order(A, hub, directed=False, return_predecessors=False)
        pos = np.empty(g.V, np.int64); pos[bo] = np.arange(len(bo))
        key = pos[src]
    elif order == "dist":
        key = csgraph.dijkstra(A, directed=False, indices=hub)[src]
    elif order in ("spt", "sptd"):
        d, pred = csgraph.dijkstra(A, directed=False, indices=hub, return_predecessors=True)
        children = [[] for _ in range(g.V)]
        for v in np.argsort(d):
            if pred[v] >= 0:
                children[pred[v]].append(v)
        pos = np.empty(g.V, np.int64)
        stack, k = [hub], 0
        while stack:
            v = stack.pop()
            pos[v] = k; k += 1
            ch = children[v]
            if order == "sptd":
                ch = sorted(ch, key=lambda c: -d[c])  # nearest child first after pop
            stack.extend(ch)
        key = pos[src]
    elif order.startswith("kd"):
        nl = int(order[2:] or 16)
        lm = np.argsort(-deg, kind="stable")[:nl]
        D = csgraph.dijkstra(A, directed=False, indices=lm)[:, src].T  # [S, nl]
        def split(idx):
            if len(idx) <= 16:
                return [idx]
            X = D[idx]
            dim = int(np.argmax(X.max(0) - X.min(0)))
            o = idx[np.argsort(X[:, dim], kind="stable")]
            half = (len(o) // 2 + 15) // 16 * 16
            return split(o[:half]) + split(o[half:])
        groups = split(np.arange(len(src)))
        key = np.empty(len(src)); k = 0
        for gi, grp in enumerate(sorted(groups, key=lambda g_: D[g_, 0].mean())):
            key[grp] = gi
    elif order == "rand":
        key = np.random.default_rng(0).random(len(src))
    src = src[np.argsort(key, kind="stable")]
    print("order", order, "hub", hub, "deg", deg[hub], flush=True)
eng = Engine(g)
ref = None
for v in variants:
    eng.set_variant(v)
    for d in deltas:
        eng.set_delta(d)
        t = eng.compute(src[:256], hosts)
        ms = []
        for _ in range(2):
            t0 = time.perf_counter()
            t = eng.compute(src, hosts, flags=SHDR_TIMING)
            ms.append(eng.timing().get('routes_pass', sum(eng.timing().values())))
        key = np.argsort(src, kind='stable')
        lat_sorted = t.lat[key]
        if ref is None:
            ref = lat_sorted.copy()
        same = np.array_equal(ref.view(np.uint64), lat_sorted.view(np.uint64))
        print(f"{os.environ.get('SHDR_LIB_VARIANT','prod'):6s} {order or 'sorted'} skip={os.environ.get('SHDR_DIAG_SKIP','0')} {wl} S={len(src)} variant={v} delta={d} kernel_ms={min(ms):.1f} same={same}", flush=True)
