"""GPU parity of the drop-in routing API (include/shd_topology.h) against the
oracle, through Shadow's own call sequence: topology_new -> topology_attach (per
host) -> topology_getReliability / topology_getLatency / topology_isRoutable.

What is checked, per reference behaviour:
  * values: complete branch = direct edge (shd-topology.c:941-979), otherwise
    shortest path + ordered epilogue (:663-773), bit-exact vs the oracle;
  * cache history: for undirected graphs a miss on (s,d) answers from a
    revealed (d,s) (:1001-1004), so the reversed-path value comes back;
  * the min-latency upcall (:602-613): worker_updateMinTimeJump receives the
    running minimum over every path stored so far, only when it drops;
  * detach: a detached address is not routable (:1296-1303, :1046-1054).
"""
import numpy as np
import pytest

from oracle import py_oracle as po
from shadow_amd import topology as top
from shadow_amd.routes import Graph
from tests.util import bits, write_graphml

pytestmark = pytest.mark.gpu


def _attach_hosts(t, n, seed):
    hosts = []
    rnd = top.Random(seed)
    for i in range(n):
        a = top.Address(f"11.0.{i // 250}.{i % 250 + 1}", f"host{i}")
        t.attach(a, rnd)
        v = t.vertex_of(a)
        assert v >= 0
        hosts.append((a, v))
    return hosts


class Expected:
    """The reference's lazily filled path cache, replayed on oracle tables."""

    def __init__(self, lat, rel, rmin, index, complete, directed):
        self.lat, self.rel, self.rmin, self.index = lat, rel, rmin, index
        self.complete, self.directed = complete, directed
        self.revealed = set()
        self.minimum = 0.0
        self.upcalls = []

    def _key(self, s, d):
        return (s, d) if self.complete else s

    def query(self, s, d):
        i, j = self.index[s], self.index[d]
        if self._key(s, d) in self.revealed:
            return self.lat[i, j], self.rel[i, j]
        if not self.directed and self._key(d, s) in self.revealed:
            return self.lat[j, i], self.rel[j, i]
        self.revealed.add(self._key(s, d))
        m = self.lat[i, j] if self.complete else self.rmin[i]
        if self.minimum == 0 or m < self.minimum:
            self.minimum = m
            self.upcalls.append(m)
        return self.lat[i, j], self.rel[i, j]


def _replay(t, hosts, exp, pairs):
    top.reset_min_time_jump()
    for a, b in pairs:
        (sa, sv), (da, dv) = hosts[a], hosts[b]
        el, er = exp.query(sv, dv)
        # Shadow's worker_sendPacket asks reliability first, then latency (shd-worker.c:238,246)
        r = t.get_reliability(sa, da)
        lt = t.get_latency(sa, da)
        assert bits(np.float64(r)) == bits(np.float64(er)), (a, b)
        assert bits(np.float64(lt)) == bits(np.float64(el)), (a, b)
        assert t.is_routable(sa, da)
    assert top.min_time_jump_calls() == len(exp.upcalls)
    if exp.upcalls:
        assert top.last_min_time_jump() == exp.upcalls[-1]
    assert t.minimum_path_latency == exp.minimum


def _tables(og, verts, mode):
    lat, rel, _, rmin = og.routes(verts, verts, mode, threads=8)
    index = {int(v): i for i, v in enumerate(verts)}
    return lat, rel, rmin, index


def test_dropin_sssp_branch(tmp_path):
    g = Graph.generate("ba", 3000, 3, 5)
    ef, et, lat, lo, vl = g.export()
    p = tmp_path / "ba3000.graphml.xml"
    write_graphml(p, g.V, ef, et, lat, lo, vl)
    t = top.Topology.new(str(p))
    assert t is not None and not t.is_complete and not t.is_directed
    hosts = _attach_hosts(t, 300, seed=7)
    verts = np.array(sorted({v for _, v in hosts}), np.int32)
    og = po.OracleGraph(g.V, ef, et, lat, lo, vl)
    exp = Expected(*_tables(og, verts, po.MODE_CANONICAL), complete=False, directed=False)
    rng = np.random.default_rng(3)
    pairs = [tuple(x) for x in rng.integers(0, len(hosts), size=(2000, 2))]
    _replay(t, hosts, exp, pairs)
    # detach: no longer routable, -1 from every query (shd-topology.c:1052,1062)
    a0, _ = hosts[0]
    t.detach(a0)
    assert t.get_latency(a0, hosts[1][0]) == -1.0
    assert t.get_reliability(hosts[1][0], a0) == -1.0
    assert not t.is_routable(a0, hosts[1][0])
    t.free()


def test_dropin_complete_branch(topo_paths):
    t = top.Topology.new(topo_paths["full"])
    assert t is not None and t.is_complete
    hosts = _attach_hosts(t, 400, seed=1)
    g = Graph.load_graphml(topo_paths["full"])
    og = po.OracleGraph.from_graph(g)
    verts = np.array(sorted({v for _, v in hosts}), np.int32)
    exp = Expected(*_tables(og, verts, po.MODE_COMPLETE), complete=True, directed=False)
    rng = np.random.default_rng(11)
    pairs = [tuple(x) for x in rng.integers(0, len(hosts), size=(3000, 2))]
    _replay(t, hosts, exp, pairs)
    t.free()


def test_dropin_simple_topology_known_answers(topo_paths):
    """topology.simple: lat (0,0)=(1,1)=20, (0,1)=50, rel 1."""
    t = top.Topology.new(topo_paths["simple"])
    rnd = top.Random(1)
    a = top.Address("11.0.0.1", "a")
    b = top.Address("11.0.0.2", "b")
    t.attach(a, rnd)
    t.attach(b, rnd)
    va, vb = t.vertex_of(a), t.vertex_of(b)
    want = {(0, 0): 20.0, (1, 1): 20.0, (0, 1): 50.0, (1, 0): 50.0}
    assert t.get_latency(a, b) == want[(va, vb)]
    assert t.get_reliability(a, b) == 1.0
    assert t.get_latency(a, a) == 20.0
    t.free()
