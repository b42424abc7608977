"""Throughput of the offline complete-topology precompute.

cfg4 graph (BA n=100000 m=3 seed 1) with P seeded points of interest:
  * engine time of the P x P path metrics (SHDR_PATH_JITTER) vs the plain route table,
  * native GraphML write of the complete graph (P(P+1)/2 edges) to local disk,
  * the reference tool's own per-source cost (networkx single_source_dijkstra_path +
    the per-path loop of compute-topology-paths.py:13-36) on a few sources, one core.
Usage: python tools/complete_bench.py [P] [out_dir]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from shadow_amd import complete_topology as ct  # noqa: E402
from shadow_amd._lib import SHDR_PATH_JITTER, SHDR_TIMING  # noqa: E402
from shadow_amd.routes import Engine, Graph  # noqa: E402


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    out_dir = sys.argv[2] if len(sys.argv) > 2 else "/tmp"
    g = Graph.generate("ba", 100_000, 3, 1)
    pois = np.sort(np.random.default_rng(1).permutation(g.V)[:P]).astype(np.int32)
    eng = Engine(g, device=0)
    eng.compute(pois[:64], pois)  # warm-up (landmarks, arena)
    res = {}
    for name, fl in (("route_table", 0), ("path_jitter", SHDR_PATH_JITTER)):
        t0 = time.perf_counter()
        t = eng.compute(pois, pois, flags=fl | SHDR_TIMING)
        dt = time.perf_counter() - t0
        res[name] = (dt, eng.timing().get('routes_pass', sum(eng.timing().values())))
        print(f"{name}: {dt:.3f} s wall (incl. D2H of {2 * P * P * 8 / 1e9:.1f} GB), kernels {res[name][1]:.1f} ms",
              flush=True)
    lat, jit = t.lat, t.rel
    path = os.path.join(out_dir, f"complete_{P}.graphml.xml")
    t0 = time.perf_counter()
    ct.write_complete(g, pois, lat, jit, path)
    dt = time.perf_counter() - t0
    size = os.path.getsize(path)
    print(f"write: {dt:.2f} s, {P * (P + 1) // 2} edges, {size / 1e9:.2f} GB ({size / dt / 1e9:.2f} GB/s)", flush=True)
    os.unlink(path)
    # the reference tool's per-source cost (networkx), one core
    import networkx as nx
    ef, et, el, _, _ = g.export()
    G = nx.Graph()
    for a, b, l in zip(ef.tolist(), et.tolist(), el.tolist()):
        if a != b:
            G.add_edge(a, b, latency=l, jitter=0.0, weight=l)
    pset = set(pois.tolist())
    n = 3
    t0 = time.perf_counter()
    for s in pois[:n].tolist():
        paths = nx.single_source_dijkstra_path(G, s)
        for d, p in paths.items():
            if d not in pset or len(p) <= 1:
                continue
            sum(G[p[i]][p[i + 1]]["latency"] for i in range(len(p) - 1))
            sum(G[p[i]][p[i + 1]]["jitter"] for i in range(len(p) - 1))
    per = (time.perf_counter() - t0) / n
    print(f"reference tool (networkx, 1 core): {per:.2f} s/source -> {per * P / 3600:.2f} core-hours for P={P}; "
          f"GPU path metrics {res['path_jitter'][0]:.2f} s", flush=True)


if __name__ == "__main__":
    main()
