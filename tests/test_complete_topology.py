"""Offline complete-topology precompute against the networkx
restatement of compute-topology-paths.py (oracle/complete_topology.py).

CPU tests drive the native GraphML writer with tables the oracle computed, and the
point-of-interest selection; the GPU tests run the whole tool (engine with
SHDR_PATH_JITTER + writer) and feed its output back into the simulator's
complete-graph branch.
"""
import math

import networkx as nx
import numpy as np
import pytest

from oracle import complete_topology as oc
from shadow_amd import complete_topology as ct
from shadow_amd._lib import ShdrError
from shadow_amd.routes import Graph
from tests.util import bits, write_graphml


def sparse_topology(tmp_path, V=150, extra=200, seed=5, directed=False, zero_edges=0):
    rng = np.random.default_rng(seed)
    ef = list(range(1, V))
    et = [int(rng.integers(0, v)) for v in range(1, V)]
    seen = {(min(a, b), max(a, b)) for a, b in zip(ef, et)}
    while len(ef) < V - 1 + extra:
        a, b = (int(x) for x in rng.integers(0, V, 2))
        if a == b or (min(a, b), max(a, b)) in seen:
            continue
        seen.add((min(a, b), max(a, b)))
        ef.append(a)
        et.append(b)
    if directed:  # strongly connected: add every reverse arc too
        ef, et = ef + et, et + ef
    E = len(ef)
    lat = rng.uniform(1, 100, E)
    lat[:zero_edges] = 0.0
    jit = rng.uniform(0, 5, E)
    types = [rng.choice(["relay", "server", "client", "client", "pop"]) for _ in range(V)]
    geos = [rng.choice(["US", "DE", "FR", "CN", "BR"]) for _ in range(V)]
    p = tmp_path / f"sparse_{seed}_{int(directed)}.graphml.xml"
    write_graphml(p, V, np.array(ef), np.array(et), lat, rng.uniform(0, 0.01, E), rng.uniform(0, 0.02, V),
                  directed=directed, types=types, geocodes=geos, jitter=jit)
    return str(p)


def oracle_tables(G, ids):
    """Row i = the oracle's path metrics from ids[i] (NaN where unreachable)."""
    for s, d in G.edges():
        G[s][d]["weight"] = float(G[s][d]["latency"])
    P = len(ids)
    lat = np.full((P, P), np.nan)
    jit = np.full((P, P), np.nan)
    col = {n: j for j, n in enumerate(ids)}
    for i, s in enumerate(ids):
        for d, (l, j) in oc.path_metrics(G, s, set(ids)).items():
            lat[i, col[d]] = l
            jit[i, col[d]] = j
    return lat, jit


def assert_same_graph(got: nx.Graph, want: nx.Graph, exact=True):
    assert set(got.nodes) == set(want.nodes)
    for n in want.nodes:
        for k, v in want.nodes[n].items():
            assert got.nodes[n][k] == v, (n, k)
    assert got.number_of_edges() == want.number_of_edges()
    for s, d, a in want.edges(data=True):
        b = got[s][d]
        for k in ("latency", "jitter", "packetloss"):
            if exact:
                assert bits(b[k]) == bits(a[k]), (s, d, k, b[k], a[k])
            else:
                assert math.isclose(b[k], a[k], rel_tol=1e-12), (s, d, k)


@pytest.mark.parametrize("directed", [False, True])
def test_writer_matches_tool_output(tmp_path, directed):
    path = sparse_topology(tmp_path, directed=directed)
    g = Graph.load_graphml(path)
    G = nx.read_graphml(path)
    pois = ct.select_pois(g, sample=30, seed=2)
    ids = [g.vertex_str("id", int(v)) for v in pois]
    lat, jit = oracle_tables(G, ids)
    out = tmp_path / "complete.graphml.xml"
    ct.write_complete(g, pois, lat, jit, str(out))
    want = oc.complete_topology(nx.read_graphml(path), ids)
    got = nx.read_graphml(str(out))
    assert not got.is_directed()
    assert_same_graph(got, want)
    # the written file is a complete topology for the simulator's loader
    h = Graph.load_graphml(str(out))
    info = h.check()
    assert h.V == len(pois) and info.is_complete and info.is_connected


def test_writer_repairs_zero_latency(tmp_path):
    path = sparse_topology(tmp_path, V=60, extra=40, zero_edges=12, seed=9)
    g = Graph.load_graphml(path)
    pois = np.arange(g.V, dtype=np.int32)
    ids = [g.vertex_str("id", int(v)) for v in pois]
    lat, jit = oracle_tables(nx.read_graphml(path), ids)
    assert (lat == 0.0).any()
    out = tmp_path / "complete.graphml.xml"
    ct.write_complete(g, pois, lat, jit, str(out))
    want = oc.complete_topology(nx.read_graphml(path), ids)
    # the substituted mean is summed in a different edge order: last-ulp freedom there only
    assert_same_graph(nx.read_graphml(str(out)), want, exact=False)
    got = nx.read_graphml(str(out))
    assert min(a["latency"] for _, _, a in got.edges(data=True)) > 0.0


def test_writer_rejects_disconnected_and_duplicates(tmp_path):
    path = sparse_topology(tmp_path, V=20, extra=5)
    g = Graph.load_graphml(path)
    pois = np.arange(4, dtype=np.int32)
    lat = np.full((4, 4), np.nan)
    np.fill_diagonal(lat, 5.0)
    lat[0, 1] = lat[1, 0] = 3.0
    with pytest.raises(ShdrError, match="not connected"):
        ct.write_complete(g, pois, lat, np.zeros((4, 4)), str(tmp_path / "x.xml"))
    with pytest.raises(ShdrError, match="duplicate"):
        ct.write_complete(g, np.array([1, 1], np.int32), np.ones((2, 2)), np.zeros((2, 2)), str(tmp_path / "y.xml"))


def test_select_pois(tmp_path):
    path = sparse_topology(tmp_path, V=300, extra=100, seed=11)
    g = Graph.load_graphml(path)
    typ = [g.vertex_str("type", v) for v in range(g.V)]
    geo = [g.vertex_str("geocode", v) for v in range(g.V)]
    pois = ct.select_pois(g, sample=10, seed=3)
    s = set(pois.tolist())
    assert list(pois) == sorted(s)
    assert all(v in s for v in range(g.V) if typ[v] in ("relay", "server"))
    assert not any(typ[v] == "pop" for v in s)
    clients = [v for v in s if typ[v] == "client"]
    assert 10 <= len(clients) <= 10 + 5
    # every geocode that has a client is represented
    assert {geo[v] for v in range(g.V) if typ[v] == "client"} == {geo[v] for v in clients}
    assert np.array_equal(pois, ct.select_pois(g, sample=10, seed=3))
    # a sample larger than the population takes every client
    allc = ct.select_pois(g, sample=10**6, seed=3)
    assert sum(typ[v] == "client" for v in allc) == sum(t == "client" for t in typ)


@pytest.mark.gpu
@pytest.mark.parametrize("directed", [False, True])
def test_gpu_complete_topology_matches_oracle(tmp_path, directed):
    path = sparse_topology(tmp_path, V=400, extra=600, seed=21, directed=directed)
    g = Graph.load_graphml(path)
    pois = ct.select_pois(g, sample=60, seed=4)
    ids = [g.vertex_str("id", int(v)) for v in pois]
    lat, jit = ct.path_tables(g, pois)
    olat, ojit = oracle_tables(nx.read_graphml(path), ids)
    assert np.array_equal(bits(lat), bits(olat))
    assert np.array_equal(bits(jit), bits(ojit))
    out = tmp_path / "complete.graphml.xml"
    ct.main([path, str(out), "--sample", "60", "--seed", "4"])
    assert_same_graph(nx.read_graphml(str(out)), oc.complete_topology(nx.read_graphml(path), ids))


@pytest.mark.gpu
def test_gpu_complete_topology_feeds_direct_branch(tmp_path):
    """Pipeline closure: the precomputed file, served by the engine's complete branch,
    answers every pair with the precomputed latency."""
    from shadow_amd.routes import Engine
    path = sparse_topology(tmp_path, V=300, extra=400, seed=23)
    out = tmp_path / "complete.graphml.xml"
    ct.main([path, str(out), "--all"])
    h = Graph.load_graphml(str(out))
    assert h.check().is_complete
    T = np.arange(h.V, dtype=np.int32)
    t = Engine(h, device=0).compute(T, T)
    G = nx.read_graphml(str(out))
    ids = [h.vertex_str("id", int(v)) for v in T]
    for i in range(0, h.V, 7):
        for j in range(0, h.V, 5):
            want = 0.0 + G[ids[i]][ids[j]]["latency"]
            assert bits(t.lat[i, j]) == bits(want)
