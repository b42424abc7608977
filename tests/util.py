"""Test helpers: GraphML writer for synthetic topologies and fixture loaders."""
from __future__ import annotations

import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def write_graphml(path, V, efrom, eto, lat, loss, vloss, directed=False, ips=None, types=None, geocodes=None,
                  jitter=None):
    """Shadow-style GraphML (the key layout of resource/topology*.graphml.xml)."""
    lines = ['<?xml version="1.0" encoding="utf-8"?><graphml xmlns="http://graphml.graphdrawing.org/xmlns">',
             '  <key attr.name="packetloss" attr.type="double" for="edge" id="d9" />',
             '  <key attr.name="jitter" attr.type="double" for="edge" id="d8" />',
             '  <key attr.name="latency" attr.type="double" for="edge" id="d7" />',
             '  <key attr.name="type" attr.type="string" for="node" id="d5" />',
             '  <key attr.name="bandwidthup" attr.type="int" for="node" id="d4" />',
             '  <key attr.name="bandwidthdown" attr.type="int" for="node" id="d3" />',
             '  <key attr.name="geocode" attr.type="string" for="node" id="d2" />',
             '  <key attr.name="ip" attr.type="string" for="node" id="d1" />',
             '  <key attr.name="packetloss" attr.type="double" for="node" id="d0" />',
             f'  <graph edgedefault="{"directed" if directed else "undirected"}">']
    for v in range(V):
        ip = ips[v] if ips is not None else "0.0.0.0"
        ty = types[v] if types is not None else "net"
        gc = geocodes[v] if geocodes is not None else "US"
        lines.append(f'    <node id="poi-{v + 1}"><data key="d0">{float(vloss[v])!r}</data><data key="d1">{ip}</data>'
                     f'<data key="d2">{gc}</data><data key="d3">10240</data><data key="d4">10240</data>'
                     f'<data key="d5">{ty}</data></node>')
    jitter = np.zeros(len(efrom)) if jitter is None else jitter
    for a, b, l, p, j in zip(efrom, eto, lat, loss, jitter):
        lines.append(f'    <edge source="poi-{int(a) + 1}" target="poi-{int(b) + 1}"><data key="d7">{float(l)!r}</data>'
                     f'<data key="d8">{float(j)!r}</data><data key="d9">{float(p)!r}</data></edge>')
    lines += ["  </graph>", "</graphml>"]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def load_sssp(kind):
    return dict(np.load(os.path.join(GOLDEN, f"sssp_{kind}.npz")))


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)
