"""Offline complete-topology precompute, restated — TEST INFRASTRUCTURE ONLY.

Checker for shadow_amd/complete_topology.py (GPU engine with SHDR_PATH_JITTER +
shdr_write_complete_graphml). Restates
/root/reference/src/tools/topology/compute-topology-paths.py (Python 2,
networkx 1.x; not runnable here) on networkx 3.4, run
sequentially (one worker, results applied in source order):
  path metrics     worker                  :13-36  (single_source_dijkstra_path,
                                                    latency sum, mean jitter, 5.0/0.0 self rule)
  pair edges       thread                  :38-44  (nx.Graph.add_edge: later source overwrites)
  zero repair      ensure_nonzero_latency  :96-112
  node copy        main                    :153-160
networkx's Dijkstra is an implementation independent of the GPU engine; the
pairs compared are those whose shortest path is unique (random f64 latencies).
"""
from __future__ import annotations

import networkx as nx


def path_metrics(G, src, pois):
    """worker(): {dst: (latency, jitter)} for every reachable dst in pois."""
    paths = nx.single_source_dijkstra_path(G, src, weight="weight")
    d = {}
    for dst, p in paths.items():
        if dst not in pois:
            continue
        if len(p) <= 1:
            lat, jit = [5.0], [0.0]
        else:
            lat, jit = [], []
            for i in range(len(p) - 1):
                e = G[p[i]][p[i + 1]]
                lat.append(float(e["latency"]))
                jit.append(float(e["jitter"]))
        d[dst] = (float(sum(lat)), float(sum(jit) / float(len(jit))))
    return d


def ensure_nonzero_latency(G):
    lintra, linter, zeros = [], [], []
    for s, d in G.edges():
        lat = G[s][d]["latency"]
        if lat <= 0.0:
            zeros.append((s, d))
        elif s == d:
            lintra.append(lat)
        else:
            linter.append(lat)
    if zeros:  # (the tool divides unconditionally and fails on an empty list)
        mi = float(sum(lintra)) / float(len(lintra))
        me = float(sum(linter)) / float(len(linter))
        for s, d in zeros:
            G[s][d]["latency"] = mi if s == d else me
    return G


def complete_topology(G, pois_in_order):
    """-> nx.Graph: the tool's output graph for sources run in the given order."""
    for s, d in G.edges():
        G[s][d]["weight"] = float(G[s][d]["latency"])
    pois = set(pois_in_order)
    Gnew = nx.Graph()
    for nid in pois_in_order:
        Gnew.add_node(nid)
        for attr, val in G.nodes[nid].items():
            Gnew.nodes[nid][attr] = val
    for src in pois_in_order:
        for dst, (lat, jit) in path_metrics(G, src, pois).items():
            Gnew.add_edge(src, dst, latency=lat, jitter=jit, packetloss=0.0)
    return ensure_nonzero_latency(Gnew)
