"""Pin the CPU oracle (oracle/shd_oracle.c) against golden vectors before it is
trusted as the GPU checker:
  * known answers of the reference's own test-config topologies (refcfg.json);
  * complete-branch tables of the bundled topologies, computed independently
    (xml.etree + Python floats, tests/golden/make_golden.py);
  * networkx shortest-path distances and, for unique-path pairs, the ordered
    epilogue along networkx's path;
  * scheduler-window and packet-delay arithmetic (shd-master.c:118-144,
    shd-worker.c:247).
"""
import json
import os

import numpy as np
import pytest

from oracle import py_oracle as po
from shadow_amd.routes import Graph


def oracle_from_text(text):
    return po.OracleGraph.from_graph(Graph.parse_graphml(text))


def test_refcfg_known_answers(golden_dir):
    cases = json.load(open(os.path.join(golden_dir, "refcfg.json")))
    assert len(cases) >= 4
    seen = set()
    for c in cases:
        og = oracle_from_text(c["graphml"])
        assert og.is_complete()  # one vertex + self-loop is "complete" (:201)
        for s, t, lat, rel in c["complete_pairs"]:
            got = og.lookup_path(s, t)
            assert got == (lat, rel), (c["files"], got, lat, rel)
            seen.add((lat, rel))
    # the values SURVEY §8(c) reads off the configs
    assert (50.0, 1.0) in seen and (50.0, 0.75) in seen and (50.0, -99.0) in seen
    assert (50.0, 0.95) in seen and (1.0, 1.0) in seen


def test_simple_topology_known_answers(topo_paths):
    og = po.OracleGraph.from_graph(Graph.load_graphml(topo_paths["simple"]))
    assert og.is_complete()
    assert og.lookup_path(0, 0) == (20.0, 1.0)
    assert og.lookup_path(1, 1) == (20.0, 1.0)
    assert og.lookup_path(0, 1) == (50.0, 1.0)
    assert og.lookup_path(1, 0) == (50.0, 1.0)


@pytest.mark.parametrize("name", ["simple", "full", "plab"])
def test_bundled_direct_tables(name, topo_paths, golden_dir):
    z = np.load(os.path.join(golden_dir, f"direct_{name}.npz"))
    g = Graph.load_graphml(topo_paths[name])
    assert g.V == int(z["V"]) and g.E == int(z["E"])
    ids = [g.vertex_str("id", v) for v in range(g.V)]
    assert ids == list(z["ids"])
    og = po.OracleGraph.from_graph(g)
    assert og.is_complete()
    V = g.V
    src = np.arange(V, dtype=np.int32)
    lat, rel, hops, rmin = og.routes(src, src, po.MODE_COMPLETE)
    assert np.array_equal(lat.view(np.uint64), z["lat"].view(np.uint64))
    assert np.array_equal(rel.view(np.uint64), z["rel"].view(np.uint64))
    assert np.array_equal(rmin, lat.min(axis=1))


def _fixture(golden_dir, kind):
    z = dict(np.load(os.path.join(golden_dir, f"sssp_{kind}.npz")))
    og = po.OracleGraph(int(z["V"]), z["efrom"], z["eto"], z["elat"], z["eloss"], z["vloss"], bool(z["directed"]))
    return z, og


@pytest.mark.parametrize("kind", ["ba2k", "dir800", "grid_ties"])
def test_dijkstra_matches_networkx(kind, golden_dir):
    z, og = _fixture(golden_dir, kind)
    assert not og.is_complete()
    for i, s in enumerate(z["sources"][:12]):
        d, pe = og.dijkstra(int(s))
        nd = z["dist"][i]
        assert np.array_equal(d.view(np.uint64), nd.view(np.uint64)), kind  # bitwise


@pytest.mark.parametrize("kind", ["ba2k", "dir800", "grid_ties"])
@pytest.mark.parametrize("mode", [po.MODE_IGRAPH, po.MODE_CANONICAL])
def test_routes_unique_pairs_bitexact(kind, mode, golden_dir):
    z, og = _fixture(golden_dir, kind)
    src, dst = z["sources"], z["targets"]
    lat, rel, hops, rmin = og.routes(src, dst, mode)
    u = z["unique"]
    assert u.sum() > 0
    assert np.array_equal(lat[u].view(np.uint64), z["lat"][u].view(np.uint64))
    assert np.array_equal(rel[u].view(np.uint64), z["rel"][u].view(np.uint64))
    assert np.array_equal(hops[u], z["hops"][u])
    # every pair: latency equals the shortest distance (self pair: self-loop)
    off = src[:, None] != dst[None, :]
    assert np.array_equal(lat[off].view(np.uint64), z["dist"][off].view(np.uint64))
    assert np.array_equal(rmin, np.nanmin(lat, axis=1))


def test_tie_pairs_canonical_paths_are_tight(golden_dir):
    z, og = _fixture(golden_dir, "grid_ties")
    for s in z["sources"][:6]:
        d, _ = og.dijkstra(int(s))
        pred, nt = og.canonical_pred(int(s), d)
        for v in range(og.V):
            if v == s:
                assert pred[v] == -1
                continue
            u = pred[v]
            assert u >= 0 and nt[v] >= 1
            e = og.get_eid(u, v)
            assert d[u] + z["elat"][e] == d[v]
        # canonical = the tight predecessor with the smallest distance, then the
        # minimum index (vectorised over all arcs)
        a = np.concatenate([z["efrom"], z["eto"]])
        b = np.concatenate([z["eto"], z["efrom"]])
        w = np.concatenate([z["elat"], z["elat"]])
        tight = (a != b) & (b != s) & (d[a] + w == d[b])
        mind = np.full(og.V, np.inf)
        np.minimum.at(mind, b[tight], d[a[tight]])
        at = tight & (d[a] == mind[b])
        best = np.full(og.V, np.iinfo(np.int32).max)
        np.minimum.at(best, b[at], a[at])
        has = best != np.iinfo(np.int32).max
        assert np.array_equal(pred[has], best[has])
        # and it is igraph's parent (first tight relaxation in pop order of the
        # restated heap Dijkstra) wherever the smallest distance is not tied
        _, pe = og.dijkstra(int(s))
        par = np.full(og.V, -1)
        hv = np.nonzero(pe >= 0)[0]
        ea, eb = z["efrom"][pe[hv]], z["eto"][pe[hv]]
        par[hv] = np.where(ea == hv, eb, ea)
        uv = np.unique(np.stack([a[at], b[at]], 1), axis=0)
        sure = np.bincount(uv[:, 1], minlength=og.V) == 1
        assert sure.sum() > 0 and np.array_equal(pred[sure], par[sure])


def test_unique_mask_matches_fixture(golden_dir):
    z, og = _fixture(golden_dir, "grid_ties")
    for i, s in enumerate(z["sources"][:8]):
        d, _ = og.dijkstra(int(s))
        pred, nt = og.canonical_pred(int(s), d)
        assert np.array_equal(po.unique_mask(pred, nt, d, int(s)), z["unique"][i])


def test_window_and_delay_semantics():
    # shd-master.c:138 truncates ms before scaling; 0 -> 10 ms default (:123)
    assert po.window_ns(5.0) == 5_000_000
    assert po.window_ns(5.9) == 5_000_000
    assert po.window_ns(0.7) == 10_000_000
    assert po.window_ns(5.0, runahead_ns=7_000_000) == 7_000_000
    assert po.delay_ns(20.0) == 20_000_000
    assert po.delay_ns(0.0000001) == 1
