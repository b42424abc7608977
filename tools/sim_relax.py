#!/usr/bin/env python3
"""Input for tools/sim_relax.c (relaxation-policy model; experiments only).

usage: python tools/sim_relax.py <cfg5|cfg4|gen:kind:n:hosts> <out.bin> [buckets=8]
Writes the bench workload's graph (undirected CSR without self-loops, each
vertex's arcs sorted by weight), pendant flags, the engine's auto window
(delta = mean_w * min(1, (1e5 / vexp)^0.42)) and `buckets` seeded K=16 source
groups of the landmark kd grouping the engine uses (routes.hip kd_groups)."""
import os
import struct
import sys

import numpy as np
import scipy.sparse as sp
from scipy.sparse.csgraph import dijkstra

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

K = 16


def main():
    wl, out = sys.argv[1], sys.argv[2]
    nbk = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    if wl.startswith("gen:"):
        from shadow_amd.routes import Graph
        _, kind, n, nh = wl.split(":")
        g = Graph.generate(kind, int(n), 3, 1)
        hosts = np.sort(np.random.default_rng(1).permutation(g.V)[:int(nh)]).astype(np.int32)
    else:
        g, hosts, _, _ = bench.make_workload(wl)
    ef, et, lat, _, _ = g.export()
    V = g.V
    keep = ef != et
    a, b, w = ef[keep].astype(np.int64), et[keep].astype(np.int64), lat[keep]
    src = np.concatenate([a, b]); dst = np.concatenate([b, a]); ww = np.concatenate([w, w])
    order = np.lexsort((ww, src))
    src, dst, ww = src[order], dst[order], ww[order]
    rowptr = np.zeros(V + 1, np.int64)
    np.add.at(rowptr, src + 1, 1)
    rowptr = np.cumsum(rowptr)
    # pendant: every arc joins one single neighbour
    deg = np.diff(rowptr)
    nb_min = np.full(V, -1, np.int64); nb_max = np.full(V, -1, np.int64)
    np.maximum.at(nb_max, src, dst)
    nb_min[:] = V
    np.minimum.at(nb_min, src, dst)
    pend = ((deg > 0) & (nb_min == nb_max)).astype(np.uint8)
    vexp = V - int(pend.sum())
    mean_w = float(ww.mean())
    delta = mean_w * min(1.0, (1e5 / vexp) ** 0.42)
    # landmarks: 4 highest-degree vertices (ties by index), distances to every vertex
    lm = np.lexsort((np.arange(V), -deg))[:4]
    M = sp.csr_matrix((ww, dst.astype(np.int32), rowptr), shape=(V, V))
    ld = dijkstra(M, directed=True, indices=lm)
    ld[~np.isfinite(ld)] = 0.0
    # kd groups over the hosts (recursive median split along the widest coordinate)
    S = len(hosts)
    gs = [min(S, i) for i in range(0, S + K, K)]
    gs = sorted(set(gs))
    idx = np.arange(S)

    def kd(g0, g1):
        if g1 - g0 <= 1:
            return
        lo, hi = gs[g0], gs[g1]
        sel = hosts[idx[lo:hi]]
        widths = [ld[k, sel].max() - ld[k, sel].min() for k in range(4)]
        k = int(np.argmax(widths))
        o = np.argsort(ld[k, sel], kind="stable")
        idx[lo:hi] = idx[lo:hi][o]
        gm = g0 + (g1 - g0 + 1) // 2
        kd(g0, gm)
        kd(gm, g1)

    sys.setrecursionlimit(10000)
    kd(0, len(gs) - 1)
    ng = len(gs) - 1
    pick = np.random.default_rng(7).choice(ng - 1, nbk, replace=False)  # full groups only
    bsrc = np.full((nbk, K), -1, np.int32)
    for i, gi in enumerate(pick):
        s = hosts[idx[gs[gi]:gs[gi + 1]]]
        bsrc[i, :len(s)] = s
    with open(out, "wb") as f:
        f.write(struct.pack("<iqdi", V, len(dst), delta, nbk))
        f.write(rowptr.astype(np.int64).tobytes())
        f.write(dst.astype(np.int32).tobytes())
        f.write(ww.astype(np.float64).tobytes())
        f.write(pend.tobytes())
        f.write(bsrc.tobytes())
    print(f"V={V} A={len(dst)} vexp={vexp} delta={delta:.3f} buckets={nbk} hubs(deg>=64)={(deg >= 64).sum()}")


if __name__ == "__main__":
    main()
