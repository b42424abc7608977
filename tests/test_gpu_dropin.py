"""GPU parity of the drop-in routing API (include/shd_topology.h) against the
oracle, through Shadow's own call sequence: topology_new -> topology_attach (per
host) -> topology_getReliability / topology_getLatency / topology_isRoutable.

What is checked, per reference behaviour:
  * values: complete branch = direct edge (shd-topology.c:941-979), otherwise
    shortest path + ordered epilogue (:663-773), bit-exact vs the oracle;
  * cache history: for undirected graphs a miss on (s,d) answers from a
    revealed (d,s) (:1001-1004), so the reversed-path value comes back;
  * the min-latency upcall (:602-613): worker_updateMinTimeJump receives the
    running minimum over every path stored so far, only when it drops. The
    reference stores a computed row target by target (in g_hash_table_get_values
    order, :791-797, :914-929) and may upcall several times within one row; the
    drop-in upcalls once per revealed row with the row minimum, which is the
    value the reference's last upcall for that row carries, so the master's
    nextMinJumpTime (shd-master.c:135-138, last call wins) is the same after
    every row. The tests assert a strictly decreasing sequence whose values are
    revealed-row minima and whose last value is the reference's running minimum;
  * a row revealed before a target was attached does not hold that target: a
    later query to it misses and recomputes the row (:775-939);
  * detach: a detached address is not routable (:1296-1303, :1046-1054);
  * several engines (SHDR_NUM_GPUS, rows split across them) and concurrent
    queries from many worker threads (shd-worker.c:238,246).
"""
import threading

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
    """The reference's lazily filled path cache, replayed on oracle tables over
    every host vertex. SSSP rows are computed over the targets attached at the
    time (`attached`), so a row holds exactly those columns; a source's cache
    only gains entries, so a pair is cached once ANY computation of its row had
    the target (g_hash_table_replace per stored target, shd-topology.c:575-600).
    A pair whose path fails (the self pair of a vertex without a self-loop:
    get_eid(s, s) fails, :733-739) is never stored, and a row computation with a
    failed target returns allSuccess = FALSE (:910-938), which fails the query
    that triggered it (-1, :1018-1035) although every other target was stored.
    `self_loop` = the vertices with a self-loop (None: every vertex has one)."""

    def __init__(self, lat, rel, rmin, index, complete, directed, self_loop=None):
        self.lat, self.rel, self.rmin, self.index = lat, rel, rmin, index
        self.complete, self.directed = complete, directed
        self.self_loop = self_loop
        self.revealed = {}  # complete: {(s, d)}; SSSP: {s: frozenset(targets)}
        self.attached = frozenset(index)
        self.minimum = 0.0
        self.row_minima = []  # every value the reference's last upcall of a row could carry, in order
        self.failed_queries = 0

    def _ok(self, s, d):  # the pair's path can be stored
        return s != d or self.self_loop is None or s in self.self_loop

    def _has(self, s, d):
        if self.complete:
            return (s, d) in self.revealed
        return d in self.revealed.get(s, ()) and self._ok(s, d)

    def query(self, s, d):
        i, j = self.index[s], self.index[d]
        if self._has(s, d):
            return self.lat[i, j], self.rel[i, j]
        if not self.directed and self._has(d, s):
            return self.lat[j, i], self.rel[j, i]
        ok = True
        if self.complete:
            m = self.lat[i, j]
            if m == m:
                self.revealed[(s, d)] = True
            ok = m == m
        else:
            self.revealed[s] = self.revealed.get(s, frozenset()) | self.attached
            cols = [self.index[v] for v in self.attached]
            m = np.nanmin(self.lat[i, cols])
            ok = self._ok(s, s)  # the source is always one of the row's targets (:791-797)
        if m == m and (self.minimum == 0 or m < self.minimum):
            self.minimum = m
            self.row_minima.append(m)
        if not ok:
            self.failed_queries += 1
            return -1.0, -1.0
        return self.lat[i, j], self.rel[i, j]


def check_upcalls(t, exp):
    """Strictly decreasing; each value a revealed row's (pair's) minimum at the
    moment it undercut the running minimum; the last one the reference's
    running minimum (what shd-master.c:135-138 ends up holding)."""
    hist = top.min_time_jump_history()
    assert all(b < a for a, b in zip(hist, hist[1:])), hist
    assert hist == exp.row_minima
    if exp.row_minima:
        assert top.last_min_time_jump() == exp.minimum
    assert t.minimum_path_latency == exp.minimum


def _replay(t, hosts, exp, pairs, reset=True):
    if reset:
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
    check_upcalls(t, exp)


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


def _ba_topology(tmp_path, n=3000, seed=5):
    g = Graph.generate("ba", n, 3, seed)
    ef, et, lat, lo, vl = g.export()
    p = tmp_path / f"ba{n}.graphml.xml"
    write_graphml(p, g.V, ef, et, lat, lo, vl)
    return g, po.OracleGraph(g.V, ef, et, lat, lo, vl), str(p)


def test_dropin_attach_after_reveal(tmp_path):
    """Rows revealed before more hosts attach do not hold the new targets: the
    first query to a new target misses, the row is recomputed over every host
    attached by then and its minimum reaches the tracker (shd-topology.c:775-939,
    :602-613); reverse-cache answers follow the same rule."""
    g, og, path = _ba_topology(tmp_path)
    t = top.Topology.new(path)
    rnd = top.Random(3)
    hosts = []
    for i in range(260):
        a = top.Address(f"11.0.{i // 250}.{i % 250 + 1}", f"host{i}")
        hosts.append(a)
    first, later = hosts[:200], hosts[200:]
    for a in first:
        t.attach(a, rnd)
    top.reset_min_time_jump()
    verts_first = {t.vertex_of(a) for a in first}
    rng = np.random.default_rng(5)
    pairs1 = [tuple(x) for x in rng.integers(0, len(first), size=(400, 2))]
    # attach the rest, then query old/new mixes
    results1 = [(t.get_reliability(first[a], first[b]), t.get_latency(first[a], first[b])) for a, b in pairs1]
    for a in later:
        t.attach(a, rnd)
    verts_all = {t.vertex_of(a) for a in hosts}
    assert len(verts_all) > len(verts_first)
    allv = np.array(sorted(verts_all), np.int32)
    lat, rel, _, rmin = og.routes(allv, allv, po.MODE_CANONICAL, threads=8)
    index = {int(v): i for i, v in enumerate(allv)}
    exp = Expected(lat, rel, rmin, index, complete=False, directed=False)
    exp.attached = frozenset(verts_first)
    vid = [t.vertex_of(a) for a in hosts]
    for (a, b), (r, lt) in zip(pairs1, results1):
        el, er = exp.query(vid[a], vid[b])
        assert bits(np.float64(r)) == bits(np.float64(er)) and bits(np.float64(lt)) == bits(np.float64(el))
    exp.attached = frozenset(verts_all)
    pairs2 = [tuple(x) for x in rng.integers(0, len(hosts), size=(600, 2))]
    pairs2 += [(a, 200 + k) for k, a in enumerate(range(0, 60))]  # old rows -> new targets
    for a, b in pairs2:
        el, er = exp.query(vid[a], vid[b])
        r = t.get_reliability(hosts[a], hosts[b])
        lt = t.get_latency(hosts[a], hosts[b])
        assert bits(np.float64(r)) == bits(np.float64(er)), (a, b)
        assert bits(np.float64(lt)) == bits(np.float64(el)), (a, b)
    check_upcalls(t, exp)
    t.free()


def test_dropin_failed_rows_without_self_loops(tmp_path):
    """Attached vertices without a self-loop (reference semantics, shd-topology.c
    :663-773, :775-939, :982-1044): the query whose miss computes such a source's
    row returns -1 (the self pair fails get_eid, so allSuccess is FALSE and the
    stored pair is not re-read), while the row's other pairs are stored and later
    queries from that source hit; (s, s) is never stored, so every query of it
    misses, recomputes the row over the targets attached at that time (revealing
    newly attached ones, with their upcall) and returns -1 again. Replayed against
    the Expected model, bit-exact, through an attach between the query phases and
    a reverse-cache (undirected) lookup on every pair. The continuation after the
    failed query is the reference's default (Release, -DNDEBUG) build: error() logs
    and returns there (shd-logger.c:209-213 calls utility_assert, empty without
    DEBUG, shd-utility.h:12-23; CMakeLists.txt:101-112); a SHADOW_DEBUG build would
    abort at the first failure instead."""
    g = Graph.generate("ba", 3000, 3, 12)
    ef, et, lat, lo, vl = g.export()
    rng = np.random.default_rng(12)
    loops = np.flatnonzero(ef == et)
    drop = set(rng.choice(loops, len(loops) // 3, replace=False).tolist())  # a third of the vertices lose theirs
    keep = np.array([e for e in range(len(ef)) if e not in drop])
    ef, et, lat, lo = ef[keep], et[keep], lat[keep], lo[keep]
    self_loop = frozenset(int(a) for a, b in zip(ef, et) if a == b)
    p = tmp_path / "ba3000_partial_loops.graphml.xml"
    write_graphml(p, g.V, ef, et, lat, lo, vl)
    t = top.Topology.new(str(p))
    assert t is not None and not t.is_complete
    rnd = top.Random(21)
    addrs = [top.Address(f"11.0.{i // 250}.{i % 250 + 1}", f"host{i}") for i in range(240)]
    first, later = addrs[:180], addrs[180:]
    for a in first:
        t.attach(a, rnd)
    og = po.OracleGraph(g.V, ef, et, lat, lo, vl)
    top.reset_min_time_jump()
    # phase 1 over the first 180 hosts; phase 2 after attaching the rest
    rng2 = np.random.default_rng(13)
    pairs1 = [tuple(x) for x in rng2.integers(0, len(first), size=(700, 2))]
    pairs1 += [(a, a) for a in range(0, 60)] + [(a, (a + 7) % 180) for a in range(0, 60)]
    got1 = [(t.get_reliability(addrs[a], addrs[b]), t.get_latency(addrs[a], addrs[b])) for a, b in pairs1]
    vid_first = [t.vertex_of(a) for a in first]
    for a in later:
        t.attach(a, rnd)
    vid = [t.vertex_of(a) for a in addrs]
    assert vid[:180] == vid_first
    allv = np.array(sorted(set(vid)), np.int32)
    assert any(v not in self_loop for v in allv) and any(v in self_loop for v in allv)
    L, R, _, rmin = og.routes(allv, allv, po.MODE_CANONICAL, threads=8)
    index = {int(v): i for i, v in enumerate(allv)}
    exp = Expected(L, R, rmin, index, complete=False, directed=False, self_loop=self_loop)
    exp.attached = frozenset(vid[:180])

    def check(pairs, got):
        for (a, b), (r, lt) in zip(pairs, got):
            # Shadow asks reliability then latency (shd-worker.c:238,246): two queries
            er = exp.query(vid[a], vid[b])[1]
            el = exp.query(vid[a], vid[b])[0]
            assert bits(np.float64(r)) == bits(np.float64(er)), (a, b, r, er)
            assert bits(np.float64(lt)) == bits(np.float64(el)), (a, b, lt, el)

    check(pairs1, got1)
    n_failed_1 = exp.failed_queries
    exp.attached = frozenset(vid)
    pairs2 = [tuple(x) for x in rng2.integers(0, len(addrs), size=(700, 2))]
    pairs2 += [(a, a) for a in range(0, 60)] + [(a, 180 + a) for a in range(0, 60)]  # self pairs, old rows -> new hosts
    got2 = [(t.get_reliability(addrs[a], addrs[b]), t.get_latency(addrs[a], addrs[b])) for a, b in pairs2]
    check(pairs2, got2)
    assert n_failed_1 > 0 and exp.failed_queries > n_failed_1  # the semantics were exercised
    check_upcalls(t, exp)
    t.free()


def _all_pairs(t, hosts):
    n = len(hosts)
    lat = np.empty((n, n))
    rel = np.empty((n, n))
    for i, (a, _) in enumerate(hosts):
        for j, (b, _) in enumerate(hosts):
            rel[i, j] = t.get_reliability(a, b)
            lat[i, j] = t.get_latency(a, b)
    return lat, rel


def test_dropin_multi_engine_row_split(tmp_path, monkeypatch):
    """SHDR_NUM_GPUS=3 engines (placed on the visible devices round-robin by the
    test switch SHDR_ENGINES_SHARE_DEVICES) each compute a third of the rows:
    every answer and the upcall sequence equal the one-engine drop-in's."""
    g, og, path = _ba_topology(tmp_path, 2000, 9)
    out = {}
    for n in ("1", "3"):
        monkeypatch.setenv("SHDR_NUM_GPUS", n)
        monkeypatch.setenv("SHDR_ENGINES_SHARE_DEVICES", "1")
        t = top.Topology.new(path)
        hosts = _attach_hosts(t, 150, seed=4)
        top.reset_min_time_jump()
        lat, rel = _all_pairs(t, hosts)
        out[n] = (lat, rel, top.min_time_jump_history(), t.minimum_path_latency)
        verts = np.array(sorted({v for _, v in hosts}), np.int32)
        t.free()
    a, b = out["1"], out["3"]
    assert np.array_equal(bits(a[0]), bits(b[0])) and np.array_equal(bits(a[1]), bits(b[1]))
    assert a[2] == b[2] and a[3] == b[3]
    lat, _, _, rmin = og.routes(verts, verts, po.MODE_CANONICAL, threads=8)
    assert b[3] == rmin.min()


def test_dropin_multi_engine_complete_plab(topo_paths, monkeypatch):
    """BASELINE config 3 through the drop-in: the PlanetLab map (complete) with
    SHDR_NUM_GPUS=3 engines each serving a block of the rows answers every pair
    of 303 attached hosts exactly as one engine does, with the same upcalls, and
    the direct-edge values equal the oracle's complete branch (:941-979)."""
    out = {}
    for n in ("1", "3"):
        monkeypatch.setenv("SHDR_NUM_GPUS", n)
        monkeypatch.setenv("SHDR_ENGINES_SHARE_DEVICES", "1")
        t = top.Topology.new(topo_paths["plab"])
        assert t is not None and t.is_complete
        hosts = _attach_hosts(t, 303, seed=3)
        top.reset_min_time_jump()
        lat, rel = _all_pairs(t, hosts)
        out[n] = (lat, rel, top.min_time_jump_history(), t.minimum_path_latency)
        t.free()
    a, b = out["1"], out["3"]
    assert np.array_equal(bits(a[0]), bits(b[0])) and np.array_equal(bits(a[1]), bits(b[1]))
    assert a[2] == b[2] and a[3] == b[3]
    g = Graph.load_graphml(topo_paths["plab"])
    og = po.OracleGraph.from_graph(g)
    t = top.Topology.new(topo_paths["plab"])
    hosts = _attach_hosts(t, 303, seed=3)
    t.free()
    verts = np.array([v for _, v in hosts], np.int32)
    lat_o, rel_o, _, _ = og.routes(verts, verts, po.MODE_COMPLETE)
    assert np.array_equal(bits(b[0]), bits(lat_o)) and np.array_equal(bits(b[1]), bits(rel_o))


def test_dropin_concurrent_queries(tmp_path):
    """16 worker threads attach concurrently (each host with its own Random, as
    host_boot seeds it), then issue interleaved getReliability/getLatency while
    the first query builds the table: every answer is a value the reference's
    history allows (the forward row, or the reverse row if it was revealed
    first, :1001-1004), and once every row is revealed the last upcall equals
    the minimum over all rows."""
    g, og, path = _ba_topology(tmp_path, 3000, 6)
    t = top.Topology.new(path)
    n = 320
    addrs = [top.Address(f"11.0.{i // 250}.{i % 250 + 1}", f"host{i}") for i in range(n)]
    rnds = [top.Random(1000 + i) for i in range(n)]
    nth = 16
    barrier = threading.Barrier(nth)

    def attach(k):
        barrier.wait()
        for i in range(k, n, nth):
            t.attach(addrs[i], rnds[i])

    th = [threading.Thread(target=attach, args=(k,)) for k in range(nth)]
    [x.start() for x in th]
    [x.join() for x in th]
    vid = [t.vertex_of(a) for a in addrs]
    ref = top.Topology.new(path)  # sequential attach: same per-host Random -> same vertices
    for i in range(n):
        ref.attach(addrs[i], top.Random(1000 + i))
    assert vid == [ref.vertex_of(a) for a in addrs]
    ref.free()
    verts = np.array(sorted(set(vid)), np.int32)
    lat, rel, _, rmin = og.routes(verts, verts, po.MODE_CANONICAL, threads=8)
    index = {int(v): i for i, v in enumerate(verts)}
    top.reset_min_time_jump()
    errors = []

    def worker(k):
        rng = np.random.default_rng(100 + k)
        barrier.wait()
        for a, b in rng.integers(0, n, size=(1500, 2)):
            r = t.get_reliability(addrs[a], addrs[b])
            lt = t.get_latency(addrs[a], addrs[b])
            i, j = index[vid[a]], index[vid[b]]
            # each call answers from the forward row or the reverse row; between the two
            # calls another thread may reveal row a (reverse -> forward), never the
            # other way round (a revealed row stays revealed)
            r_f, r_r = bits(np.float64(r)) == bits(rel[i, j]), bits(np.float64(r)) == bits(rel[j, i])
            l_f, l_r = bits(np.float64(lt)) == bits(lat[i, j]), bits(np.float64(lt)) == bits(lat[j, i])
            if not (r_f or r_r) or not (l_f or l_r) or (r_f and not r_r and l_r and not l_f):
                errors.append((a, b, lt, r))

    th = [threading.Thread(target=worker, args=(k,)) for k in range(nth)]
    [x.start() for x in th]
    [x.join() for x in th]
    assert not errors, errors[:5]
    hist = top.min_time_jump_history()
    assert hist and all(y < x for x, y in zip(hist, hist[1:]))
    assert all(h in set(rmin.tolist()) for h in hist)
    for a in addrs:  # reveal every row (a self query is never a reverse hit)
        t.get_latency(a, a)
    assert top.last_min_time_jump() == rmin.min() == t.minimum_path_latency
    t.free()


def _replay_record(path, nhosts, seed, pairs_seed, npairs, late=0):
    """Attach nhosts (the last `late` of them after the first queries), replay
    reliability + latency queries, return (answers, upcall history, minimum,
    table blocks)."""
    t = top.Topology.new(path)
    rnd = top.Random(seed)
    addrs = [top.Address(f"11.0.{i // 250}.{i % 250 + 1}", f"host{i}") for i in range(nhosts)]
    for a in addrs[:nhosts - late]:
        t.attach(a, rnd)
    top.reset_min_time_jump()
    rng = np.random.default_rng(pairs_seed)
    ans = []

    def run(n, hi):
        for a, b in rng.integers(0, hi, size=(n, 2)):
            ans.append((t.get_reliability(addrs[a], addrs[b]), t.get_latency(addrs[a], addrs[b])))

    run(npairs, nhosts - late)
    blocks_early = t.table_blocks()
    if late:
        for a in addrs[nhosts - late:]:
            t.attach(a, rnd)
        run(npairs, nhosts)
    out = (np.array(ans), top.min_time_jump_history(), t.minimum_path_latency, blocks_early)
    t.free()
    return out


@pytest.mark.parametrize("kind", ["sssp", "complete"])
def test_dropin_row_block_mode(tmp_path, topo_paths, monkeypatch, kind):
    """Row-block mode (SHDR_TABLE_BLOCK_ROWS; chosen automatically when the whole
    table would exceed SHDR_TABLE_HOST_FRAC of host RAM): rows are computed a
    block at a time, on the first query that needs one of them, so host memory
    follows the rows actually used as the reference's per-source rows do
    (shd-topology.c:775-939). Answers, the min-latency upcall sequence and the
    final minimum must be identical to the whole-table mode's, through an
    attach-after-reveal epoch change, with one engine and with two."""
    if kind == "sssp":
        _, _, path = _ba_topology(tmp_path, 3000, 8)
        nh = 240
    else:
        path = topo_paths["full"]
        nh = 300
    res = {}
    for mode, rows, gpus in (("whole", None, "1"), ("blocks", "16", "1"), ("blocks2", "24", "2")):
        monkeypatch.setenv("SHDR_NUM_GPUS", gpus)
        monkeypatch.setenv("SHDR_ENGINES_SHARE_DEVICES", "1")
        if rows:
            monkeypatch.setenv("SHDR_TABLE_BLOCK_ROWS", rows)
        else:
            monkeypatch.delenv("SHDR_TABLE_BLOCK_ROWS", raising=False)
        res[mode] = _replay_record(path, nh, 5, 9, 300, late=40)
    w = res["whole"]
    assert w[3][0] == 1 and w[3][2] == 1  # one block, computed at the first query
    for mode in ("blocks", "blocks2"):
        b = res[mode]
        assert np.array_equal(bits(b[0]), bits(w[0])), mode
        assert b[1] == w[1] and b[2] == w[2], mode
        nblk, rows_per, done = b[3]
        assert nblk > 1 and done <= nblk, b[3]
    # lazily: a few queries from one source compute only that source's block
    monkeypatch.setenv("SHDR_NUM_GPUS", "1")
    monkeypatch.setenv("SHDR_TABLE_BLOCK_ROWS", "16")
    t = top.Topology.new(path)
    hosts = _attach_hosts(t, nh, seed=5)
    for k in range(1, 20):
        t.get_latency(hosts[0][0], hosts[k][0])
    nblk, _, done = t.table_blocks()
    assert nblk > 4 and done == 1, (nblk, done)
    times = t.last_compute_times()
    assert times["block_rows"] <= 16 and times["block_ms"] > 0
    t.free()
