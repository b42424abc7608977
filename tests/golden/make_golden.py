#!/usr/bin/env python3
"""Regenerate the golden fixtures under tests/golden/ (run in the dev container,
where /root/reference exists; the GPU box only reads the committed outputs).

Independent of both the product (shadow_amd/) and the C oracle: GraphML is
parsed with xml.etree, routing values are computed in Python floats (IEEE f64,
in the reference's operation order), shortest paths come from networkx 3.4.2.

Outputs
  refcfg.json           topologies embedded (CDATA) in the reference's own test
                        configs + the bundled example + the built-in --test
                        example, with the known answer for their one pair
                        (shd-topology.c:941-979 on a one-vertex self-loop graph)
  topologies/*.xz       the three bundled topologies (resource/, data)
  direct_<name>.npz     complete-branch tables (all ordered pairs) for the
                        bundled topologies: lat/rel [V,V] in igraph vertex order
  sssp_<name>.npz       shortest-path fixtures on synthetic graphs: edges,
                        sources, targets, networkx distances, unique-path mask,
                        expected lat/rel/hops for unique pairs
"""
from __future__ import annotations

import glob
import hashlib
import json
import lzma
import os
import re
import shutil
import xml.etree.ElementTree as ET

import networkx as nx
import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
NS = "{http://graphml.graphdrawing.org/xmlns}"


# ------------------------------------------------------------------ GraphML (independent reader)
def parse_graphml(text: str):
    root = ET.fromstring(text)
    keys = {}
    for k in root.iter(NS + "key"):
        keys[k.get("id")] = (k.get("attr.name"), k.get("attr.type"), k.get("for"))
    graph = root.find(NS + "graph")
    directed = graph.get("edgedefault") == "directed"
    index, ids = {}, []

    def vid(x):
        if x not in index:
            index[x] = len(ids)
            ids.append(x)
        return index[x]

    vattr, eattr, ef, et = {}, [], [], []
    for el in graph:
        if el.tag == NS + "node":
            v = vid(el.get("id"))
            d = vattr.setdefault(v, {})
            for dd in el.findall(NS + "data"):
                name, ty, _ = keys[dd.get("key")]
                d[name] = float(dd.text) if ty in ("double", "int", "float", "long") else (dd.text or "")
        elif el.tag == NS + "edge":
            a, b = vid(el.get("source")), vid(el.get("target"))
            ef.append(a)
            et.append(b)
            d = {}
            for dd in el.findall(NS + "data"):
                name, ty, _ = keys[dd.get("key")]
                d[name] = float(dd.text) if ty in ("double", "int", "float", "long") else (dd.text or "")
            eattr.append(d)
    V = len(ids)
    vloss = [vattr.get(v, {}).get("packetloss", float("nan")) for v in range(V)]
    elat = [d.get("latency", float("nan")) for d in eattr]
    eloss = [d.get("packetloss", float("nan")) for d in eattr]
    return dict(ids=ids, directed=directed, efrom=ef, eto=et, elat=elat, eloss=eloss, vloss=vloss)


def canon_map(g):
    m = {}
    for e, (a, b) in enumerate(zip(g["efrom"], g["eto"])):
        k = (a, b) if g["directed"] else (min(a, b), max(a, b))
        m.setdefault(k, e)
    return m


def lookup_path(g, cm, s, t):
    """shd-topology.c:941-979 in Python floats."""
    k = (s, t) if g["directed"] else (min(s, t), max(s, t))
    if k not in cm:
        return None
    e = cm[k]
    lat, rel = 0.0, 1.0
    rel *= 1.0 - g["vloss"][s]
    rel *= 1.0 - g["vloss"][t]
    lat += g["elat"][e]
    rel *= 1.0 - g["eloss"][e]
    return lat, rel


def epilogue(g, cm, s, path):
    """shd-topology.c:663-773 in Python floats; path = igraph vertex list."""
    lat, rel = 0.0, 1.0
    rel *= 1.0 - g["vloss"][s]
    nv = len(path)
    if nv == 0:
        lat = 1.0
    else:
        d = path[-1]
        if s != d or (s == d and nv > 2):
            rel *= 1.0 - g["vloss"][d]
        start = 0 if nv == 1 else 1
        frm = s
        for i in range(start, nv):
            to = path[i]
            k = (frm, to) if g["directed"] else (min(frm, to), max(frm, to))
            if k not in cm:
                return None
            e = cm[k]
            lat += g["elat"][e]
            rel *= 1.0 - g["eloss"][e]
            frm = to
    if lat == 0.0:
        lat = 1.0
    return lat, rel


# ------------------------------------------------------------------ 1. reference test configs
def refcfg():
    found = {}
    files = sorted(glob.glob(f"{REF}/src/test/**/*.xml", recursive=True)) + [f"{REF}/resource/examples/shadow.config.xml"]
    for f in files:
        txt = open(f).read()
        m = re.search(r"<topology><!\[CDATA\[(.*?)\]\]></topology>", txt, re.S)
        if not m:
            continue
        body = m.group(1)
        h = hashlib.sha256(body.encode()).hexdigest()[:16]
        found.setdefault(h, {"graphml": body, "files": []})["files"].append(os.path.relpath(f, REF))
    # the built-in --test example, src/main/core/support/shd-examples.c:10-50 (C string literal)
    src = open(f"{REF}/src/main/core/support/shd-examples.c").read()
    m = re.search(r"<!\[CDATA\[(.*?)\]\]>", src, re.S)
    body = m.group(1).replace('\\"', '"').replace("\\\n", "\n")
    h = hashlib.sha256(body.encode()).hexdigest()[:16]
    found.setdefault(h, {"graphml": body, "files": []})["files"].append("src/main/core/support/shd-examples.c")
    cases = []
    for h, c in sorted(found.items()):
        g = parse_graphml(c["graphml"])
        cm = canon_map(g)
        pairs = []
        for s in range(len(g["ids"])):
            for t in range(len(g["ids"])):
                r = lookup_path(g, cm, s, t)
                pairs.append([s, t, r[0], r[1]] if r else [s, t, None, None])
        cases.append({"sha": h, "files": c["files"], "graphml": c["graphml"], "V": len(g["ids"]),
                      "complete_pairs": pairs})
    json.dump(cases, open(os.path.join(OUT, "refcfg.json"), "w"), indent=1)
    print(f"refcfg.json: {len(cases)} distinct topologies from {sum(len(c['files']) for c in cases)} configs")


# ------------------------------------------------------------------ 2+3. bundled topologies
BUNDLED = {"simple": "topology.simple.graphml.xml.xz", "full": "topology.graphml.xml.xz",
           "plab": "topology.plab.graphml.xml.xz"}


def bundled():
    os.makedirs(os.path.join(OUT, "topologies"), exist_ok=True)
    for name, fn in BUNDLED.items():
        shutil.copyfile(f"{REF}/resource/{fn}", os.path.join(OUT, "topologies", fn))
        g = parse_graphml(lzma.open(f"{REF}/resource/{fn}").read().decode())
        cm = canon_map(g)
        V = len(g["ids"])
        lat = np.full((V, V), np.nan)
        rel = np.full((V, V), np.nan)
        for s in range(V):
            for t in range(V):
                r = lookup_path(g, cm, s, t)
                if r:
                    lat[s, t], rel[s, t] = r
        np.savez_compressed(os.path.join(OUT, f"direct_{name}.npz"), ids=np.array(g["ids"]), lat=lat, rel=rel,
                            V=V, E=len(g["efrom"]))
        print(f"direct_{name}.npz: V={V} E={len(g['efrom'])} nan={np.isnan(lat).sum()}")


# ------------------------------------------------------------------ 4. shortest-path fixtures
def synth(kind, seed):
    rng = np.random.default_rng(seed)
    if kind == "ba2k":
        G = nx.barabasi_albert_graph(2000, 2, seed=seed)
        edges = list(G.edges())
        V, directed = 2000, False
        lat = rng.uniform(1.0, 100.0, len(edges))
    elif kind == "dir800":
        V, directed = 800, True
        perm = rng.permutation(V)
        edges = [(int(perm[i]), int(perm[(i + 1) % V])) for i in range(V)]  # Hamiltonian cycle
        seen = set(edges)
        while len(edges) < 5 * V:
            a, b = (int(x) for x in rng.integers(0, V, 2))
            if a != b and (a, b) not in seen:
                seen.add((a, b))
                edges.append((a, b))
        lat = rng.uniform(1.0, 50.0, len(edges))
    elif kind == "grid_ties":
        n = 24
        V, directed = n * n, False
        edges = []
        for r in range(n):
            for c in range(n):
                v = r * n + c
                if c + 1 < n:
                    edges.append((v, v + 1))
                if r + 1 < n:
                    edges.append((v, v + n))
        lat = rng.integers(1, 4, len(edges)).astype(np.float64)  # integer weights: many ties
    else:
        raise ValueError(kind)
    eloss = rng.uniform(0.0, 0.01, len(edges))
    vloss = rng.uniform(0.0, 0.02, V)
    ef = [a for a, _ in edges] + list(range(V))
    et = [b for _, b in edges] + list(range(V))
    elat = list(lat) + list(rng.uniform(0.5, 5.0, V))
    elo = list(eloss) + list(rng.uniform(0.0, 0.01, V))
    return dict(ids=[f"poi-{i + 1}" for i in range(V)], directed=directed, efrom=ef, eto=et, elat=elat, eloss=elo,
                vloss=list(vloss))


def sssp_fixture(kind, seed, nsrc):
    g = synth(kind, seed)
    cm = canon_map(g)
    V = len(g["ids"])
    G = nx.DiGraph() if g["directed"] else nx.Graph()
    G.add_nodes_from(range(V))
    for e, (a, b) in enumerate(zip(g["efrom"], g["eto"])):
        if a != b:
            G.add_edge(a, b, latency=g["elat"][e])
    rng = np.random.default_rng(seed + 100)
    sources = np.sort(rng.choice(V, nsrc, replace=False)).astype(np.int32)
    targets = np.arange(V, dtype=np.int32)
    S, T = len(sources), len(targets)
    dist = np.full((S, T), np.nan)
    uniq = np.zeros((S, T), bool)
    elat = np.full((S, T), np.nan)
    erel = np.full((S, T), np.nan)
    ehops = np.full((S, T), -1, np.int32)
    # tight in-arcs for uniqueness (bitwise fl(d[u]+w) == d[v])
    inarcs = [[] for _ in range(V)]
    for e, (a, b) in enumerate(zip(g["efrom"], g["eto"])):
        if a == b:
            continue
        inarcs[b].append((a, g["elat"][e]))
        if not g["directed"]:
            inarcs[a].append((b, g["elat"][e]))
    for i, s in enumerate(sources):
        d, paths = nx.single_source_dijkstra(G, int(s), weight="latency")
        dv = np.array([d.get(v, np.nan) for v in range(V)])
        dist[i] = dv
        ntight = np.zeros(V, np.int32)
        for v in range(V):
            if v == s:
                continue
            us = {u for (u, w) in inarcs[v] if dv[u] + w == dv[v]}
            ntight[v] = len(us)
        order = np.argsort(dv)
        un = np.zeros(V, bool)
        un[s] = True
        for v in order:
            if v == s:
                continue
            p = paths[v][-2]
            un[v] = ntight[v] == 1 and un[p]
        uniq[i] = un
        for j, t in enumerate(targets):
            path = [int(s)] if t == s else [int(x) for x in paths[int(t)]]
            r = epilogue(g, cm, int(s), path)
            if r and un[t]:
                elat[i, j], erel[i, j] = r
                ehops[i, j] = 1 if len(path) == 1 else len(path) - 1
    np.savez_compressed(os.path.join(OUT, f"sssp_{kind}.npz"), V=V, directed=g["directed"],
                        efrom=np.array(g["efrom"], np.int32), eto=np.array(g["eto"], np.int32),
                        elat=np.array(g["elat"]), eloss=np.array(g["eloss"]), vloss=np.array(g["vloss"]),
                        sources=sources, targets=targets, dist=dist, unique=uniq, lat=elat, rel=erel, hops=ehops)
    print(f"sssp_{kind}.npz: V={V} E={len(g['efrom'])} S={S} unique pairs {uniq.mean():.3f}")


if __name__ == "__main__":
    refcfg()
    bundled()
    sssp_fixture("ba2k", 7, 48)
    sssp_fixture("dir800", 11, 40)
    sssp_fixture("grid_ties", 5, 24)
