"""GPU parity: the HIP engine (through the shdr_* C-ABI) against golden vectors
and the CPU oracle on the same seeded inputs.

Bar (north_star): bit-exact latency, reliability and hop count for every pair
whose shortest path is unique (and for every pair of the complete-graph
branch); on tie pairs the engine's canonical rule (minimum-index tight
predecessor) is compared bit-exactly with the oracle's canonical mode, and the
latency must equal the shortest distance.  Table-level tolerance where a
reversed fold is compared (undirected symmetry): 1e-12 relative.
"""
import json
import os

import numpy as np
import pytest

from oracle import py_oracle as po
from shadow_amd.routes import SHDR_FORCE_SSSP, SHDR_KEEP_TREES, SHDR_TIMING, Engine, Graph
from tests.util import bits, load_sssp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bundled(topo_paths):
    return {k: Graph.load_graphml(p) for k, p in topo_paths.items()}


@pytest.mark.parametrize("name", ["simple", "full", "plab"])
def test_direct_branch_bundled_bitexact(name, bundled, golden_dir):
    z = np.load(os.path.join(golden_dir, f"direct_{name}.npz"))
    g = bundled[name]
    assert g.check().is_complete
    eng = Engine(g)
    v = np.arange(g.V, dtype=np.int32)
    t = eng.compute(v, v, hops=True, flags=SHDR_TIMING)
    assert np.array_equal(bits(t.lat), bits(z["lat"]))
    assert np.array_equal(bits(t.rel), bits(z["rel"]))
    assert (t.hops == 1).all()
    assert np.array_equal(bits(t.row_min), bits(z["lat"].min(axis=1)))
    assert "k_routes_direct" in eng.timing()


def test_refcfg_topologies(golden_dir):
    for c in json.load(open(os.path.join(golden_dir, "refcfg.json"))):
        g = Graph.parse_graphml(c["graphml"])
        eng = Engine(g)
        v = np.arange(g.V, dtype=np.int32)
        t = eng.compute(v, v)
        for s, d, lat, rel in c["complete_pairs"]:
            assert t.lat[s, d] == lat and t.rel[s, d] == rel, c["files"]


def _graph_from_fixture(z):
    return Graph.from_edges(int(z["V"]), z["efrom"], z["eto"], z["elat"], z["eloss"], z["vloss"],
                            directed=bool(z["directed"]))


@pytest.mark.parametrize("kind", ["ba2k", "dir800", "grid_ties"])
def test_sssp_fixtures(kind):
    z = load_sssp(kind)
    g = _graph_from_fixture(z)
    assert not g.check().is_complete
    eng = Engine(g)
    src, dst = z["sources"], z["targets"]
    t = eng.compute(src, dst, hops=True)
    u = z["unique"]
    # unique pairs: bit-exact against the independent (networkx) golden vectors
    assert np.array_equal(bits(t.lat[u]), bits(z["lat"][u]))
    assert np.array_equal(bits(t.rel[u]), bits(z["rel"][u]))
    assert np.array_equal(t.hops[u], z["hops"][u])
    # all off-diagonal pairs: latency == shortest distance, bitwise
    off = src[:, None] != dst[None, :]
    assert np.array_equal(bits(t.lat[off]), bits(z["dist"][off]))
    # every pair (ties included): bit-exact against the oracle's canonical mode
    og = po.OracleGraph(int(z["V"]), z["efrom"], z["eto"], z["elat"], z["eloss"], z["vloss"], bool(z["directed"]))
    lat, rel, hops, rmin = og.routes(src, dst, po.MODE_CANONICAL)
    assert np.array_equal(bits(t.lat), bits(lat))
    assert np.array_equal(bits(t.rel), bits(rel))
    assert np.array_equal(t.hops, hops)
    assert np.array_equal(bits(t.row_min), bits(rmin))


@pytest.mark.parametrize("kind", ["grid_ties", "dir800", "ba2k"])
def test_chain_pass_few_targets(kind):
    """T <= V/2 runs the chain-restricted predecessor pass (only the targets'
    ancestors get predecessor entries): tie-heavy and directed graphs, every pair
    bit-exact against the oracle's canonical mode, and identical to the full pass
    (targets = all vertices) on the same columns."""
    z = load_sssp(kind)
    g = _graph_from_fixture(z)
    V = int(z["V"])
    rng = np.random.default_rng(7)
    dst = np.sort(rng.choice(V, size=max(1, V // 5), replace=False)).astype(np.int32)
    src = z["sources"]
    eng = Engine(g)
    t = eng.compute(src, dst, hops=True)
    og = po.OracleGraph(V, z["efrom"], z["eto"], z["elat"], z["eloss"], z["vloss"], bool(z["directed"]))
    lat, rel, hops, rmin = og.routes(src, dst, po.MODE_CANONICAL)
    assert np.array_equal(bits(t.lat), bits(lat))
    assert np.array_equal(bits(t.rel), bits(rel))
    assert np.array_equal(t.hops, hops)
    assert np.array_equal(bits(t.row_min), bits(rmin))
    full = eng.compute(src, np.arange(V, dtype=np.int32), hops=True)
    assert np.array_equal(bits(full.lat[:, dst]), bits(t.lat))
    assert np.array_equal(bits(full.rel[:, dst]), bits(t.rel))


@pytest.mark.parametrize("kind", ["grid_ties", "dir800"])
def test_near_bitmap_mode_fixtures(kind, monkeypatch):
    """Mode 1 on the tie-heavy and directed fixtures, every pair bit-exact."""
    monkeypatch.setenv("SHDR_PENDING_LDS", "1")
    z = load_sssp(kind)
    g = _graph_from_fixture(z)
    src, dst = z["sources"], z["targets"]
    t = Engine(g).compute(src, dst, hops=True)
    og = po.OracleGraph(int(z["V"]), z["efrom"], z["eto"], z["elat"], z["eloss"], z["vloss"], bool(z["directed"]))
    lat, rel, hops, _ = og.routes(src, dst, po.MODE_CANONICAL)
    assert np.array_equal(bits(t.lat), bits(lat))
    assert np.array_equal(bits(t.rel), bits(rel))
    assert np.array_equal(t.hops, hops)


def test_near_bitmap_mode_at_scale():
    """A graph too large for both LDS bitmaps (V = 300k) runs mode 1 by default."""
    g = Graph.generate("chunglu", 300_000, 3, 11)
    rng = np.random.default_rng(2)
    src = rng.choice(g.V, 40, replace=False).astype(np.int32)
    dst = rng.choice(g.V, 2000, replace=False).astype(np.int32)
    t = Engine(g).compute(src, dst, hops=True)
    og = po.OracleGraph.from_graph(g)
    lat, rel, hops, rmin = og.routes(src, dst, po.MODE_CANONICAL, threads=8)
    assert np.array_equal(bits(t.lat), bits(lat))
    assert np.array_equal(bits(t.rel), bits(rel))
    assert np.array_equal(t.hops, hops)
    assert np.array_equal(bits(t.row_min), bits(rmin))


def test_pred_trees_match_oracle():
    z = load_sssp("grid_ties")
    g = _graph_from_fixture(z)
    eng = Engine(g)
    src = z["sources"]
    eng.compute(src, z["targets"], flags=SHDR_KEEP_TREES)
    og = po.OracleGraph(int(z["V"]), z["efrom"], z["eto"], z["elat"], z["eloss"], z["vloss"], bool(z["directed"]))
    for i, s in enumerate(src):
        pred, dist = eng.pred_tree(i)
        d, _ = og.dijkstra(int(s))
        opred, _ = og.canonical_pred(int(s), d)
        assert np.array_equal(bits(dist), bits(d))
        assert np.array_equal(pred, opred)


def test_forced_sssp_on_complete_topology(bundled):
    """The bundled complete graphs never run Dijkstra in the reference; forcing
    the shortest-path branch on them exercises dense high-degree CSR rows."""
    g = bundled["full"]
    eng = Engine(g)
    v = np.arange(g.V, dtype=np.int32)
    t = eng.compute(v, v, hops=True, flags=SHDR_FORCE_SSSP)
    og = po.OracleGraph.from_graph(g)
    lat, rel, hops, rmin = og.routes(v, v, po.MODE_CANONICAL)
    assert np.array_equal(bits(t.lat), bits(lat))
    assert np.array_equal(bits(t.rel), bits(rel))
    assert np.array_equal(t.hops, hops)
    direct = eng.compute(v, v)
    assert (t.lat <= direct.lat).all()  # shortest <= direct edge
    assert (t.lat < direct.lat).sum() > 0


@pytest.mark.parametrize("n,m,S,T,seed", [(20000, 3, 100, 1500, 3), (5000, 2, 37, 5000, 9)])
def test_generated_ba_vs_oracle(n, m, S, T, seed):
    g = Graph.generate("ba", n, m, seed)
    eng = Engine(g)
    rng = np.random.default_rng(seed)
    src = rng.choice(n, S, replace=False).astype(np.int32)
    dst = rng.choice(n, T, replace=False).astype(np.int32)
    dst[:5] = src[:5]  # self pairs
    t = eng.compute(src, dst, hops=True)
    og = po.OracleGraph.from_graph(g)
    lat, rel, hops, rmin = og.routes(src, dst, po.MODE_CANONICAL, threads=8)
    assert np.array_equal(bits(t.lat), bits(lat))
    assert np.array_equal(bits(t.rel), bits(rel))
    assert np.array_equal(t.hops, hops)
    assert np.array_equal(bits(t.row_min), bits(rmin))


def test_chunglu_vs_oracle():
    g = Graph.generate("chunglu", 30000, 3, 5)
    info = g.check()
    assert info.is_connected and not info.is_complete
    eng = Engine(g)
    rng = np.random.default_rng(1)
    src = rng.choice(g.V, 40, replace=False).astype(np.int32)
    dst = rng.choice(g.V, 3000, replace=False).astype(np.int32)
    t = eng.compute(src, dst, hops=True)
    og = po.OracleGraph.from_graph(g)
    lat, rel, hops, rmin = og.routes(src, dst, po.MODE_CANONICAL, threads=8)
    assert np.array_equal(bits(t.lat), bits(lat))
    assert np.array_equal(bits(t.rel), bits(rel))


def test_slot_rows_reused_without_fill():
    """No per-bucket fill of the distance rows: on a strongly connected
    graph a slot's rows alternate between two encodings from bucket to bucket and
    keep the previous bucket's words. One engine computes a sequence of tables:
    more buckets than CUs (several buckets per slot), a partial bucket, a
    keep-trees call (plain encoding, trees read back) and full tables again,
    each bit-exact against the oracle."""
    g = Graph.generate("ba", 6000, 3, 21)
    assert g.check().is_connected
    eng = Engine(g)
    og = po.OracleGraph.from_graph(g)
    rng = np.random.default_rng(4)
    dst = rng.choice(g.V, 400, replace=False).astype(np.int32)
    everyone = rng.permutation(g.V).astype(np.int32)
    calls = [(everyone, 0), (everyone[:37], 0), (everyone[100:164], SHDR_KEEP_TREES), (everyone[::-1].copy(), 0),
             (everyone[:5000], 0)]
    for src, flags in calls:
        t = eng.compute(src, dst, hops=True, flags=flags)
        lat, rel, hops, rmin = og.routes(src, dst, po.MODE_CANONICAL, threads=8)
        assert np.array_equal(bits(t.lat), bits(lat)), len(src)
        assert np.array_equal(bits(t.rel), bits(rel)), len(src)
        assert np.array_equal(t.hops, hops), len(src)
        assert np.array_equal(bits(t.row_min), bits(rmin)), len(src)
        if flags:
            for i in (0, 17, 63):
                pred, dist = eng.pred_tree(i)
                d, _ = og.dijkstra(int(src[i]))
                assert np.array_equal(bits(dist), bits(d))


def test_slot_rows_reused_across_layouts(monkeypatch):
    """No-fill across layout changes on one engine: tables alternate between
    a main launch plus a concurrent half-width tail in its own arena region, a single
    launch over the whole arena, and a partial bucket, so arena regions are reused
    with another slot stride and a region's rows may hold another bucket's encoding.
    Every table is bit-exact against the oracle and the same list gives the same table
    again."""
    monkeypatch.setenv("SHDR_TAIL_MIN_WAVES", "1")
    monkeypatch.setenv("SHDR_BALANCE", "0")
    g = Graph.generate("ba", 6000, 3, 29)
    eng = Engine(g)
    og = po.OracleGraph.from_graph(g)
    rng = np.random.default_rng(8)
    dst = rng.choice(g.V, 300, replace=False).astype(np.int32)
    everyone = rng.permutation(g.V).astype(np.int32)
    seen = {}
    for n in (6000, 2000, 6000, 21, 6000, 4100, 2000):
        src = everyone[:n]
        t = eng.compute(src, dst, hops=True, flags=SHDR_TIMING)
        lat, rel, hops, rmin = og.routes(src, dst, po.MODE_CANONICAL, threads=8)
        assert np.array_equal(bits(t.lat), bits(lat)), n
        assert np.array_equal(bits(t.rel), bits(rel)), n
        assert np.array_equal(t.hops, hops), n
        assert np.array_equal(bits(t.row_min), bits(rmin)), n
        lay = eng.last_layout()
        seen.setdefault("tail" if lay["rows_main"] < n else "single", []).append((n, lay["tail_mode"]))
    assert seen.get("tail") and seen.get("single"), seen
    assert all(m == 3 for _, m in seen["tail"]), seen  # the tail rows ran inside the one launch


def test_edge_cases():
    # path graph 0-1-2-3 (undirected), self-loop only on vertex 0: a self pair
    # without a self-loop has no path (reference: get_eid error, :733-739)
    ef = np.array([0, 1, 2, 0], np.int32)
    et = np.array([1, 2, 3, 0], np.int32)
    lat = np.array([1.5, 2.25, 3.0, 0.5])
    loss = np.array([0.1, 0.2, 0.0, 0.3])
    vl = np.array([0.01, 0.0, 0.02, 0.0])
    g = Graph.from_edges(4, ef, et, lat, loss, vl)
    assert not g.check().is_complete
    eng = Engine(g)
    t = eng.compute([0, 3, 1], [0, 1, 2, 3], hops=True)
    assert t.lat[0, 0] == 0.5 and t.rel[0, 0] == (1.0 - 0.01) * (1.0 - 0.3)
    assert t.hops[0, 0] == 1
    assert t.lat[0, 3] == (1.5 + 2.25) + 3.0
    r = 1.0 * (1 - 0.01)
    r *= 1 - 0.0
    r *= 1 - 0.1
    r *= 1 - 0.2
    r *= 1 - 0.0
    assert t.rel[0, 3] == r and t.hops[0, 3] == 3
    assert np.isnan(t.lat[1, 3])  # 3 -> 3 has no self-loop
    assert t.lat[1, 0] == (3.0 + 2.25) + 1.5  # reversed fold order from source 3
    assert t.row_min[0] == 0.5
    # empty inputs
    e = eng.compute(np.zeros(0, np.int32), [0, 1])
    assert e.lat.shape == (0, 2)
    # duplicate sources and targets
    t2 = eng.compute([2, 2], [1, 1, 3])
    assert np.array_equal(bits(t2.lat[0]), bits(t2.lat[1]))


def test_long_paths_beyond_hop_stack():
    """Paths far longer than the epilogue's per-chain hop stack (14): the walk
    re-folds in chunks; both lockstep chains of a lane end at different depths."""
    rng = np.random.default_rng(12)
    n = 400
    ring = np.arange(n, dtype=np.int32)
    ef = np.concatenate([ring, ring[::50], ring])
    et = np.concatenate([(ring + 1) % n, (ring[::50] + 25) % n, ring])  # ring, a few chords, self-loops
    E = len(ef)
    lat = rng.uniform(1.0, 100.0, E)
    g = Graph.from_edges(n, ef, et, lat, rng.uniform(0, 0.01, E), rng.uniform(0, 0.02, n))
    eng = Engine(g)
    src = rng.choice(n, 40, replace=False).astype(np.int32)
    dst = np.arange(0, n, 3, dtype=np.int32)
    t = eng.compute(src, dst, hops=True)
    og = po.OracleGraph.from_graph(g)
    lat_o, rel_o, hops_o, rmin = og.routes(src, dst, po.MODE_CANONICAL)
    assert hops_o.max() > 40
    assert np.array_equal(bits(t.lat), bits(lat_o))
    assert np.array_equal(bits(t.rel), bits(rel_o))
    assert np.array_equal(t.hops, hops_o)
    assert np.array_equal(bits(t.row_min), bits(rmin))


def test_directed_asymmetry():
    # 0->1->2->0 cycle plus a shortcut 0->2: directed, strongly connected
    ef = np.array([0, 1, 2, 0, 0, 1, 2], np.int32)
    et = np.array([1, 2, 0, 2, 0, 1, 2], np.int32)
    lat = np.array([1.0, 1.0, 1.0, 5.0, 0.25, 0.25, 0.25])
    g = Graph.from_edges(3, ef, et, lat, np.zeros(7), np.zeros(3), directed=True)
    eng = Engine(g)
    t = eng.compute([0, 1, 2], [0, 1, 2], hops=True)
    assert t.lat[0, 2] == 2.0 and t.hops[0, 2] == 2
    assert t.lat[2, 0] == 1.0 and t.lat[1, 0] == 2.0


def test_large_row_count_padding():
    """S not a multiple of the bucket width, several buckets per slot."""
    g = Graph.generate("ba", 3000, 3, 21)
    eng = Engine(g)
    src = np.arange(0, 3000, 7, dtype=np.int32)  # 429 rows
    dst = np.arange(0, 3000, 3, dtype=np.int32)
    t = eng.compute(src, dst)
    og = po.OracleGraph.from_graph(g)
    lat, rel, _, _ = og.routes(src, dst, po.MODE_CANONICAL, threads=8)
    assert np.array_equal(bits(t.lat), bits(lat))
    assert np.array_equal(bits(t.rel), bits(rel))


def test_delta_independence():
    """Result must not depend on the relaxation bucket width."""
    g = Graph.generate("ba", 8000, 3, 4)
    eng = Engine(g)
    src = np.arange(0, 8000, 97, dtype=np.int32)
    dst = np.arange(0, 8000, 5, dtype=np.int32)
    ref = eng.compute(src, dst, hops=True)
    for d in (1.0, 7.5, 1e9):
        eng.set_delta(d)
        t = eng.compute(src, dst, hops=True)
        assert np.array_equal(bits(t.lat), bits(ref.lat))
        assert np.array_equal(bits(t.rel), bits(ref.rel))
        assert np.array_equal(t.hops, ref.hops)


@pytest.mark.parametrize("variant", ["4", "7"])
def test_tail_submission_order_parity(variant, monkeypatch):
    """The half-width tail rows run inside the one table launch (default, k_routes_pass:
    the first workgroups take the tail's buckets, then full-width ones; variant 4), or
    as a concurrent launch on a second stream submitted before the main launch (with
    the hold kernel in front of the main launch) or after it (SHDR_PASS=0 and
    SHDR_TAIL_FIRST=1 / 0; variant 7, whose single launch is not built, always does):
    only where the tail's buckets run changes, so every table equals the oracle's bit
    for bit. The tail is forced at 1.5 waves (SHDR_TAIL_MIN_WAVES=1)."""
    monkeypatch.setenv("SHDR_TAIL_MIN_WAVES", "1")
    monkeypatch.setenv("SHDR_BALANCE", "0")
    monkeypatch.setenv("SHDR_VARIANT", variant)
    g = Graph.generate("ba", 6000, 3, 23)
    rng = np.random.default_rng(5)
    # K = 32 buckets need 8,192 rows for one full wave: sources repeat past the graph's vertices
    src = (rng.permutation(g.V)[:6005] if variant == "4" else rng.choice(g.V, 32 * 356)).astype(np.int32)
    dst = np.arange(0, g.V, 31, dtype=np.int32)
    lat, rel, hops, rmin = po.OracleGraph.from_graph(g).routes(src, dst, po.MODE_CANONICAL, threads=8)
    for single, tf in (("1", "1"), ("0", "1"), ("0", "0")):
        monkeypatch.setenv("SHDR_PASS", single)
        monkeypatch.setenv("SHDR_TAIL_FIRST", tf)
        eng = Engine(g)
        for _ in range(2):
            t = eng.compute(src, dst, hops=True, flags=SHDR_TIMING)
            lay = eng.last_layout()
            assert lay["rows_main"] < len(src), lay
            assert lay["tail_mode"] == (3 if single == "1" and variant == "4" else 2), (single, tf, lay)
            assert ("k_routes_sssp_tail" in eng.timing()) == (lay["tail_mode"] == 2), eng.timing()
            assert np.array_equal(bits(t.lat), bits(lat)) and np.array_equal(bits(t.rel), bits(rel)), tf
            assert np.array_equal(t.hops, hops) and np.array_equal(bits(t.row_min), bits(rmin)), tf
        del eng


@pytest.mark.parametrize("tail_min_waves,balance,ctail,nsrc", [
    ("1", "0", None, 6000), (None, "0", "1", 6000), (None, "0", "1", 8832), (None, "0", None, 6000),
    (None, "1", None, 6000),
    # S % 16 != 0: the partial group is issued first (explicit bucket offsets)
    ("1", "0", None, 6005), (None, "0", "1", 8837), (None, "0", None, 6005), (None, "0", None, 3339)])
def test_tail_split_and_grouping_parity(tail_min_waves, balance, ctail, nsrc, monkeypatch):
    """S large enough for full waves of buckets plus a partial last wave: run as
    the half-width concurrent tail (forced at 1.5 waves), as a cluster tail
    (SHDR_CLUSTER_TAIL: 6,000 rows leave 119 of 256 buckets after one wave -> cl 2,
    8,832 rows leave 40 after two -> cl 4; sources repeat past the graph's 6,000
    vertices), without a tail, or balanced; landmark grouping and longest-first
    order: every row must land in its caller-order position, bit-exact against
    the oracle, and stay so when the same source list is re-run. The layout that
    ran is asserted (a cluster tail that fell back would not count)."""
    if tail_min_waves:
        monkeypatch.setenv("SHDR_TAIL_MIN_WAVES", tail_min_waves)
    if ctail:
        monkeypatch.setenv("SHDR_CLUSTER_TAIL", ctail)
    monkeypatch.setenv("SHDR_BALANCE", balance)
    g = Graph.generate("ba", 6000, 3, 17)
    eng = Engine(g)
    rng = np.random.default_rng(2)
    src = (rng.permutation(g.V)[:nsrc] if nsrc <= g.V else rng.choice(g.V, nsrc)).astype(np.int32)  # scrambled
    dst = np.arange(0, g.V, 29, dtype=np.int32)
    t = eng.compute(src, dst, hops=True)
    lay = eng.last_layout()
    if ctail:
        assert lay["tail_cluster"] >= 2 and lay["cluster_fallback"] == 0, lay
    assert lay["cluster_fallbacks_total"] == 0, lay
    og = po.OracleGraph.from_graph(g)
    lat, rel, hops, rmin = og.routes(src, dst, po.MODE_CANONICAL, threads=8)
    assert np.array_equal(bits(t.lat), bits(lat))
    assert np.array_equal(bits(t.rel), bits(rel))
    assert np.array_equal(t.hops, hops)
    assert np.array_equal(bits(t.row_min), bits(rmin))
    # the same source list again: buckets re-issued in measured-duration order (on by
    # default for launches of at most 4 waves of buckets, as here: <= 552 buckets)
    order1 = eng.row_order()
    orders = []
    for _ in range(2):
        t2 = eng.compute(src, dst, hops=True)
        orders.append(eng.row_order())
        assert np.array_equal(bits(t2.lat), bits(lat))
        assert np.array_equal(bits(t2.rel), bits(rel))
        assert np.array_equal(t2.hops, hops)
        assert np.array_equal(bits(t2.row_min), bits(rmin))
    assert sorted(order1.tolist()) == sorted(orders[0].tolist())
    if not ctail:
        assert not np.array_equal(order1, orders[0]), "measured-duration order not applied"


@pytest.mark.parametrize("variant,mode",[(4, 0), (1, 0), (6, 0), (4, 1), (6, 1), (7, 0), (7, 1), (7, 2)])
def test_pending_sets_in_global_memory(variant, mode, monkeypatch):
    """The slot byte-array pending sets (mode 0) and the near-bitmap-only mode
    (mode 1: near set in LDS, far set in slot bytes, hop stacks sharing the
    bitmap's LDS; used when both bitmaps do not fit, e.g. cfg5) give the same
    tables as the LDS bitmaps."""
    g = Graph.generate("chunglu", 7000, 3, 8)
    src = np.random.default_rng(4).choice(g.V, 300, replace=False).astype(np.int32)
    dst = np.arange(0, g.V, 11, dtype=np.int32)
    monkeypatch.setenv("SHDR_PENDING_LDS", str(mode))
    monkeypatch.setenv("SHDR_VARIANT", str(variant))
    eng = Engine(g)
    t = eng.compute(src, dst, hops=True)
    og = po.OracleGraph.from_graph(g)
    lat, rel, hops, rmin = og.routes(src, dst, po.MODE_CANONICAL, threads=8)
    assert np.array_equal(bits(t.lat), bits(lat))
    assert np.array_equal(bits(t.rel), bits(rel))
    assert np.array_equal(t.hops, hops)
    assert np.array_equal(bits(t.row_min), bits(rmin))
    # every vertex a source: more buckets than slots, so slots run several buckets
    # and the chain pass's queue bits must be back to zero for the next one
    allv = np.arange(g.V, dtype=np.int32)
    t2 = eng.compute(allv, dst)
    lat2, rel2, _, _ = og.routes(allv, dst, po.MODE_CANONICAL, threads=8)
    assert np.array_equal(bits(t2.lat), bits(lat2))
    assert np.array_equal(bits(t2.rel), bits(rel2))


@pytest.mark.parametrize("kind", ["grid_ties", "dir800"])
def test_device_numbering_independence(kind, monkeypatch):
    """The engine renumbers vertices breadth-first from the hub (routes.hip
    relabel_bfs). Tables, hop counts and predecessor trees (reported in the
    caller's numbering) must equal those of the caller's numbering, including on
    tie-heavy graphs whose canonical tie rule depends on per-vertex arc order;
    the fixture's vertices are scrambled first so the renumbering moves them."""
    z = load_sssp(kind)
    V = int(z["V"])
    newid = np.random.default_rng(5).permutation(V).astype(np.int32)
    g = Graph.from_edges(V, newid[z["efrom"]], newid[z["eto"]], z["elat"], z["eloss"],
                         z["vloss"][np.argsort(newid)], directed=bool(z["directed"]))
    src, dst = newid[z["sources"]], newid[z["targets"]]
    out = {}
    for r in ("0", "1"):
        monkeypatch.setenv("SHDR_RELABEL", r)
        eng = Engine(g)
        t = eng.compute(src, dst, hops=True, flags=SHDR_KEEP_TREES)
        out[r] = (t, [eng.pred_tree(i) for i in range(min(len(src), 8))])
    (a, pa), (b, pb) = out["0"], out["1"]
    assert np.array_equal(bits(a.lat), bits(b.lat))
    assert np.array_equal(bits(a.rel), bits(b.rel))
    assert np.array_equal(a.hops, b.hops)
    assert np.array_equal(bits(a.row_min), bits(b.row_min))
    og = po.OracleGraph(V, newid[z["efrom"]], newid[z["eto"]], z["elat"], z["eloss"],
                        z["vloss"][np.argsort(newid)], bool(z["directed"]))
    for i, ((p0, d0), (p1, d1)) in enumerate(zip(pa, pb)):
        assert np.array_equal(p0, p1) and np.array_equal(bits(d0), bits(d1))
        d, _ = og.dijkstra(int(src[i]))
        opred, _ = og.canonical_pred(int(src[i]), d)
        assert np.array_equal(bits(d1), bits(d)) and np.array_equal(p1, opred)


def test_device_numbering_disconnected(monkeypatch):
    """relabel_bfs appends the vertices its breadth-first pass from the hub does
    not reach (other components, isolated vertices) component by component:
    unreachable pairs stay NaN / -1 and every table is identical to the
    caller's numbering."""
    rng = np.random.default_rng(11)
    ef, et = [], []
    for base, n in ((0, 300), (300, 200)):  # two random trees plus chords
        for v in range(1, n):
            ef.append(base + int(rng.integers(0, v))); et.append(base + v)
        for _ in range(n):
            a, b = rng.integers(0, n, 2)
            if a != b:
                ef.append(base + int(a)); et.append(base + int(b))
    V = 501  # vertex 500 isolated
    ef, et = np.array(ef, np.int32), np.array(et, np.int32)
    perm = rng.permutation(V).astype(np.int32)
    ef, et = perm[ef], perm[et]
    E = len(ef)
    g = Graph.from_edges(V, ef, et, rng.uniform(1, 100, E), rng.uniform(0, 0.01, E), rng.uniform(0, 0.02, V))
    src = np.arange(0, V, 7, dtype=np.int32)
    dst = np.arange(0, V, 3, dtype=np.int32)
    out = {}
    for r in ("0", "1"):
        monkeypatch.setenv("SHDR_RELABEL", r)
        out[r] = Engine(g).compute(src, dst, hops=True)
    a, b = out["0"], out["1"]
    assert np.array_equal(bits(a.lat), bits(b.lat))
    assert np.array_equal(bits(a.rel), bits(b.rel))
    assert np.array_equal(a.hops, b.hops)
    assert (b.hops < 0).any() and (b.hops > 0).any()
    og = po.OracleGraph.from_graph(g)
    lat, rel, hops, _ = og.routes(src, dst, po.MODE_CANONICAL)
    assert np.array_equal(bits(b.lat), bits(lat))
    assert np.array_equal(b.hops, hops)


def test_pred_trees_follow_igraph_parents():
    """igraph's Dijkstra (strict '<', orc_dijkstra) keeps the first tight
    relaxation in heap pop order, i.e. the tight predecessor with the smallest
    distance. Wherever that smallest distance is held by ONE predecessor, the
    engine's predecessor must be igraph's parent; only equal-distance ties (heap
    order, unpinned) fall to the lowest-index rule. Checked on the integer-weight
    grid, whose tight predecessor sets are large."""
    z = load_sssp("grid_ties")
    g = _graph_from_fixture(z)
    V = int(z["V"])
    eng = Engine(g)
    src = z["sources"]
    eng.compute(src, z["targets"], flags=SHDR_KEEP_TREES)
    og = po.OracleGraph(V, z["efrom"], z["eto"], z["elat"], z["eloss"], z["vloss"], bool(z["directed"]))
    ef, et, w = z["efrom"].astype(np.int64), z["eto"].astype(np.int64), z["elat"]
    keep = ef != et
    ef, et, w = ef[keep], et[keep], w[keep]
    if not bool(z["directed"]):
        ef, et, w = np.concatenate([ef, et]), np.concatenate([et, ef]), np.concatenate([w, w])
    distinct_ties = checked = 0
    for i, s in enumerate(src):
        pred, dist = eng.pred_tree(i)
        d, pe = og.dijkstra(int(s))
        parent = np.full(V, -1, np.int64)
        has = pe >= 0
        a, b = z["efrom"][pe[has]], z["eto"][pe[has]]
        vv = np.nonzero(has)[0]
        parent[vv] = np.where(a == vv, b, a)
        tight = (d[ef] >= 0) & (d[et] >= 0) & (et != s) & (d[ef] + w == d[et])
        u, v = ef[tight], et[tight]
        uv = np.unique(np.stack([u, v], 1), axis=0)
        u, v = uv[:, 0], uv[:, 1]
        mind = np.full(V, np.inf)
        np.minimum.at(mind, v, d[u])
        at_min = d[u] == mind[v]
        nmin = np.bincount(v[at_min], minlength=V)
        ntight = np.bincount(v, minlength=V)
        sure = nmin == 1
        distinct_ties += int(((ntight > 1) & sure).sum())
        checked += int(sure.sum())
        assert np.array_equal(pred[sure], parent[sure]), i
    assert distinct_ties > 0 and checked > 0  # ties between different distances were exercised


def _bench_workload(name):
    from bench import make_workload
    g, hosts, _, _ = make_workload(name)
    return g, hosts


def _self_pair_values(g, verts):
    """Self pair of the SSSP branch: the canonical (lowest edge id) self-loop,
    lat = 0.0 + l, rel = (1.0 * (1 - p_s)) * (1 - loss); no destination loss
    (shd-topology.c:694, :709-711, :733-743)."""
    ef, et, lat, lo, vl = g.export()
    loops = np.nonzero(ef == et)[0]
    first = {}
    for e in loops[::-1]:
        first[int(ef[e])] = e
    sl = np.array([lat[first[int(v)]] for v in verts])
    sr = np.array([(1.0 * (1.0 - vl[v])) * (1.0 - lo[first[int(v)]]) for v in verts])
    return 0.0 + sl, sr


def _launch_stratified_rows(eng, S, rows, seed):
    """Caller rows to compare, drawn per launch of the last compute: half from the
    main launch, half from the tail launch (rows past last_layout rows_main in
    the engine's processing order), plus the partial group's rows when one was
    issued first. -> (rows, set of tail rows)."""
    lay = eng.last_layout()
    order = eng.row_order()
    assert len(order) == S and np.array_equal(np.sort(order), np.arange(S))
    nm = lay["rows_main"]
    rng = np.random.default_rng(seed)
    main, tail = order[:nm], order[nm:]
    k_tail = min(len(tail), rows // 2)
    pick = [rng.choice(main, rows - k_tail, replace=False)]
    if k_tail:
        pick.append(rng.choice(tail, k_tail, replace=False))
    if lay["partial_first"]:
        pick.append(order[:min(S, 16) // 2])
    return np.unique(np.concatenate(pick)), set(int(x) for x in tail)


@pytest.mark.parametrize("name,rows", [("cfg4", 64), ("cfg5", 32)])
def test_baseline_workload_full_table(name, rows):
    """BASELINE configs 4 and 5 at full size, exactly as bench.py builds them
    (BA n=1e5 / Chung-Lu n=1e6, 10k / 50k attached hosts): the WHOLE S x T table
    is computed on the GPU into HBM (cfg5: 2.5e9 pairs, 50 GB with hop counts).
    Rows are sampled per launch (main launch and the concurrent half-width tail
    launch, which takes 848 of cfg5's rows and 1,808 of cfg4's) and compared bit
    for bit with the oracle's canonical mode (lat, rel, hops, row minimum) and with
    its restated igraph Dijkstra (MODE_IGRAPH: 2-way heap, strict '<', early
    exit; shd-topology.c:866-887), which must agree bitwise on these tie-free
    tables. Every row is checked on the device for size-independent properties:
    no NaN (connected graph), row minimum == minimum of the row, self pairs ==
    the self-loop values, and the undirected table's transpose within 1e-12
    relative (reversed folds)."""
    import torch

    g, hosts = _bench_workload(name)
    S = T = len(hosts)
    eng = Engine(g)
    dev = torch.device("cuda", 0)
    lat = torch.empty((S, T), dtype=torch.float64, device=dev)
    rel = torch.empty((S, T), dtype=torch.float64, device=dev)
    hops = torch.empty((S, T), dtype=torch.int32, device=dev)
    rmin = torch.empty((S,), dtype=torch.float64, device=dev)
    eng.compute_device(hosts, hosts, lat.data_ptr(), rel.data_ptr(), rmin.data_ptr(), hops.data_ptr(),
                       stream=torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    pick, tail = _launch_stratified_rows(eng, S, rows, 20260)
    lay = eng.last_layout()
    if torch.cuda.get_device_properties(0).multi_processor_count == 256:
        assert lay["rows_main"] < S and lay["cluster"] == 1, lay  # the bench layout: main + tail launch
    assert len(tail) == S - lay["rows_main"]
    assert sum(int(p) in tail for p in pick) >= min(len(tail), rows // 2)
    og = po.OracleGraph.from_graph(g)
    threads = min(16, len(os.sched_getaffinity(0)))
    olat, orel, ohops, ormin = og.routes(hosts[pick], hosts, po.MODE_CANONICAL, threads=threads)
    ilat, irel, ihops, irmin = og.routes(hosts[pick], hosts, po.MODE_IGRAPH, threads=threads)
    for a, b in ((olat, ilat), (orel, irel), (ormin, irmin)):
        assert np.array_equal(bits(a), bits(b)), "canonical and igraph modes differ (ties) on these rows"
    assert np.array_equal(ohops, ihops)
    idx = torch.as_tensor(pick, device=dev)
    assert np.array_equal(bits(lat[idx].cpu().numpy()), bits(olat))
    assert np.array_equal(bits(rel[idx].cpu().numpy()), bits(orel))
    assert np.array_equal(hops[idx].cpu().numpy(), ohops)
    assert np.array_equal(bits(rmin[idx].cpu().numpy()), bits(ormin))
    # whole-table properties, in row blocks on the device
    sl, sr = _self_pair_values(g, hosts)
    diag = torch.arange(S, device=dev)
    assert torch.equal(lat[diag, diag].cpu(), torch.as_tensor(sl))
    assert torch.equal(rel[diag, diag].cpu(), torch.as_tensor(sr))
    blk = 2048
    for r0 in range(0, S, blk):
        L = lat[r0:r0 + blk]
        assert not torch.isnan(L).any()
        assert torch.equal(L.amin(dim=1), rmin[r0:r0 + blk])
        assert (hops[r0:r0 + blk] >= 1).all()
        for M in (lat, rel):
            a = M[r0:r0 + blk, :]
            b = M[:, r0:r0 + blk].t()
            assert ((a - b).abs() <= 1e-12 * a.abs()).all()


def test_cfg5_strong_scaling_shards():
    """BASELINE config 5 as the 8-GPU bench cuts it (bench.py rank_sources:
    Engine.partition of the 50,000 hosts into 8 parts, identical on every rank):
    two of the eight 6,250-row shards (parts 0 and 7) computed alone, as one rank
    does, with the layout the automatic wave model picks for them asserted (plain
    K=16 buckets, the partial kd group issued first, no concurrent tail, no
    cluster fallback); 16 launch-stratified rows per shard bit-exact against the
    oracle's canonical mode AND its restated igraph Dijkstra, and every row of
    the shard checked on the device (no NaN, row minimum, hop counts)."""
    import torch

    g, hosts = _bench_workload("cfg5")
    T = len(hosts)
    eng = Engine(g)
    part = eng.partition(hosts, 8)
    assert np.bincount(part, minlength=8).tolist() == [6250] * 8
    og = po.OracleGraph.from_graph(g)
    threads = min(16, len(os.sched_getaffinity(0)))
    dev = torch.device("cuda", 0)
    for p in (0, 7):
        rows = hosts[part == p]
        S = len(rows)
        lat = torch.empty((S, T), dtype=torch.float64, device=dev)
        rel = torch.empty((S, T), dtype=torch.float64, device=dev)
        hops = torch.empty((S, T), dtype=torch.int32, device=dev)
        rmin = torch.empty((S,), dtype=torch.float64, device=dev)
        for _ in range(2):  # the second pass runs in measured-duration order (<= 4 waves of buckets)
            eng.compute_device(rows, hosts, lat.data_ptr(), rel.data_ptr(), rmin.data_ptr(), hops.data_ptr(),
                               stream=torch.cuda.current_stream(dev).cuda_stream)
            torch.cuda.synchronize(dev)
        lay = eng.last_layout()
        assert lay["cluster"] == 1 and lay["cluster_fallback"] == 0 and lay["variant"] == 4, lay
        assert lay["partial_first"] == 1 and lay["rows_main"] == S, lay  # 6,250 = 390 x 16 + 10
        pick, _ = _launch_stratified_rows(eng, S, 16, 808 + p)
        for mode in (po.MODE_CANONICAL, po.MODE_IGRAPH):
            olat, orel, ohops, ormin = og.routes(rows[pick], hosts, mode, threads=threads)
            idx = torch.as_tensor(pick, device=dev)
            assert np.array_equal(bits(lat[idx].cpu().numpy()), bits(olat)), (p, mode)
            assert np.array_equal(bits(rel[idx].cpu().numpy()), bits(orel)), (p, mode)
            assert np.array_equal(hops[idx].cpu().numpy(), ohops), (p, mode)
            assert np.array_equal(bits(rmin[idx].cpu().numpy()), bits(ormin)), (p, mode)
        assert not torch.isnan(lat).any() and (hops >= 1).all()
        assert torch.equal(lat.amin(dim=1), rmin)
        del lat, rel, hops, rmin
        torch.cuda.empty_cache()


@pytest.mark.parametrize("nparts", [8, 4])
def test_cfg4_strong_scaling_shards(nparts):
    """BASELINE config 4 as the 8- and 4-GPU bench cuts it (bench.py rank_sources:
    Engine.partition of the 10,000 hosts into 1,250- / 2,500-row parts): EVERY shard
    computed alone, as one rank does, in the layout the automatic wave model picks
    for it on a 256-CU device — 3-wide PM 2 clusters (three CUs share a bucket and
    its slot, cross-CU barriers every round) — asserted with no cluster fallback;
    16 rows per shard bit-exact against the oracle's canonical mode AND its restated
    igraph Dijkstra, and every row of every shard checked on the device (no NaN,
    row minimum, hop counts). Two passes per shard: the second reuses the slots'
    rows and runs in measured-duration order."""
    import torch

    g, hosts = _bench_workload("cfg4")
    T = len(hosts)
    eng = Engine(g)
    part = eng.partition(hosts, nparts)
    assert np.bincount(part, minlength=nparts).tolist() == [T // nparts] * nparts
    og = po.OracleGraph.from_graph(g)
    threads = min(16, len(os.sched_getaffinity(0)))
    dev = torch.device("cuda", 0)
    full_chip = torch.cuda.get_device_properties(0).multi_processor_count == 256
    S = T // nparts
    lat = torch.empty((S, T), dtype=torch.float64, device=dev)
    rel = torch.empty((S, T), dtype=torch.float64, device=dev)
    hops = torch.empty((S, T), dtype=torch.int32, device=dev)
    rmin = torch.empty((S,), dtype=torch.float64, device=dev)
    for p in range(nparts):
        rows = hosts[part == p]
        for _ in range(2):
            eng.compute_device(rows, hosts, lat.data_ptr(), rel.data_ptr(), rmin.data_ptr(), hops.data_ptr(),
                               stream=torch.cuda.current_stream(dev).cuda_stream)
            torch.cuda.synchronize(dev)
            lay = eng.last_layout()
            assert lay["cluster_fallback"] == 0 and lay["cluster_fallbacks_total"] == 0, lay
            if full_chip:
                assert lay["cluster"] == 3 and lay["variant"] == 4, lay  # the wave model's layout
        pick = np.random.default_rng(404 + p).choice(S, 16, replace=False)
        idx = torch.as_tensor(pick, device=dev)
        for mode in (po.MODE_CANONICAL, po.MODE_IGRAPH):
            olat, orel, ohops, ormin = og.routes(rows[pick], hosts, mode, threads=threads)
            assert np.array_equal(bits(lat[idx].cpu().numpy()), bits(olat)), (p, mode)
            assert np.array_equal(bits(rel[idx].cpu().numpy()), bits(orel)), (p, mode)
            assert np.array_equal(hops[idx].cpu().numpy(), ohops), (p, mode)
            assert np.array_equal(bits(rmin[idx].cpu().numpy()), bits(ormin)), (p, mode)
        assert not torch.isnan(lat).any() and (hops >= 1).all()
        assert torch.equal(lat.amin(dim=1), rmin)


@pytest.mark.parametrize("directed", [False, True])
def test_pendant_vertices_skip_relaxation(directed, monkeypatch):
    """Pendant vertices (every arc joins one neighbour: the Chung-Lu graphs'
    1-degree fringe, ~20 % of cfg5) never enter a pending set and a pendant
    source relaxes its arcs at bucket start (routes.hip DevGraph::vexp). Tables
    and trees must equal those with the skip disabled, and the oracle's, with
    pendant sources and targets in the mix."""
    rng = np.random.default_rng(8)
    base = Graph.generate("chunglu", 6000, 3, 12)
    ef, et, lat, lo, vl = base.export()
    V = base.V
    loops = ef == et
    deg = np.bincount(np.concatenate([ef[~loops], et[~loops]]), minlength=V)
    pend = np.nonzero(deg == 1)[0]
    assert len(pend) > 300
    if directed:  # both orientations of every non-loop edge, plus one-way spokes
        ef2 = np.concatenate([ef[~loops], et[~loops], ef[loops]])
        et2 = np.concatenate([et[~loops], ef[~loops], et[loops]])
        lat2 = np.concatenate([lat[~loops], lat[~loops] * 1.5, lat[loops]])
        lo2 = np.concatenate([lo[~loops], lo[~loops], lo[loops]])
        g = Graph.from_edges(V, ef2, et2, lat2, lo2, vl, directed=True)
    else:
        g = base
    src = np.concatenate([rng.choice(pend, 40, replace=False), rng.choice(V, 60, replace=False)]).astype(np.int32)
    dst = np.unique(np.concatenate([rng.choice(pend, 200, replace=False), rng.choice(V, 600, replace=False)]))
    dst = dst.astype(np.int32)
    out = {}
    for skip in ("1", "0"):
        monkeypatch.setenv("SHDR_PENDANT_SKIP", skip)
        eng = Engine(g)
        t = eng.compute(src, dst, hops=True, flags=SHDR_KEEP_TREES)
        out[skip] = (t, [eng.pred_tree(i) for i in (0, 1, 50)])
    (a, ta), (b, tb) = out["1"], out["0"]
    assert np.array_equal(bits(a.lat), bits(b.lat)) and np.array_equal(bits(a.rel), bits(b.rel))
    assert np.array_equal(a.hops, b.hops) and np.array_equal(bits(a.row_min), bits(b.row_min))
    for (p0, d0), (p1, d1) in zip(ta, tb):
        assert np.array_equal(p0, p1) and np.array_equal(bits(d0), bits(d1))
    og = po.OracleGraph.from_graph(g)
    lat_o, rel_o, hops_o, rmin_o = og.routes(src, dst, po.MODE_CANONICAL, threads=8)
    assert np.array_equal(bits(a.lat), bits(lat_o)) and np.array_equal(bits(a.rel), bits(rel_o))
    assert np.array_equal(a.hops, hops_o) and np.array_equal(bits(a.row_min), bits(rmin_o))
    # grouped, many-bucket run (landmark pre-pass, chain pass) with pendant rows
    allsrc = np.concatenate([pend[:500], np.arange(0, V, 7)]).astype(np.int32)
    monkeypatch.setenv("SHDR_PENDANT_SKIP", "1")
    t2 = Engine(g).compute(allsrc, dst)
    lat2, rel2, _, _ = og.routes(allsrc, dst, po.MODE_CANONICAL, threads=8)
    assert np.array_equal(bits(t2.lat), bits(lat2)) and np.array_equal(bits(t2.rel), bits(rel2))



@pytest.mark.parametrize("variant", ["4", "6"])
@pytest.mark.parametrize("S", [40, 300, 1250, 5000])
def test_balanced_buckets_small_shards(variant, S, monkeypatch):
    """Balanced bucket layout (routes.hip group_starts): S rows become whole waves
    of buckets holding f or f+1 sources (strong-scaling shards: fewer rows than
    K x CUs, buckets of 1-2 sources, uneven sizes); every row in its caller
    position, bit-exact, also when re-run in measured-duration order."""
    monkeypatch.setenv("SHDR_VARIANT", variant)
    g = Graph.generate("chunglu", 12000, 3, 19)
    src = np.random.default_rng(S).choice(g.V, S, replace=False).astype(np.int32)
    dst = np.arange(0, g.V, 17, dtype=np.int32)
    eng = Engine(g)
    og = po.OracleGraph.from_graph(g)
    lat, rel, hops, rmin = og.routes(src, dst, po.MODE_CANONICAL, threads=8)
    for _ in range(2):
        t = eng.compute(src, dst, hops=True)
        assert np.array_equal(bits(t.lat), bits(lat)) and np.array_equal(bits(t.rel), bits(rel))
        assert np.array_equal(t.hops, hops) and np.array_equal(bits(t.row_min), bits(rmin))


def test_partition_balanced_deterministic():
    """shdr_engine_partition: part sizes S/N or S/N + 1 (larger first), the same
    split from every engine of the graph (ranks agree without communicating),
    and the parts' rows computed separately equal the whole table's rows."""
    g = Graph.generate("chunglu", 20000, 3, 2)
    hosts = np.sort(np.random.default_rng(3).choice(g.V, 3001, replace=False)).astype(np.int32)
    e1, e2 = Engine(g), Engine(g)
    p1 = e1.partition(hosts, 8)
    p2 = e2.partition(hosts, 8)
    assert np.array_equal(p1, p2)
    assert list(np.bincount(p1, minlength=8)) == [376] * 1 + [375] * 7
    dst = hosts[::7]
    full = e1.compute(hosts, dst)
    for p in range(8):
        t = e2.compute(hosts[p1 == p], dst)
        assert np.array_equal(bits(t.lat), bits(full.lat[p1 == p])) and np.array_equal(bits(t.rel),
                                                                                      bits(full.rel[p1 == p]))
    assert np.array_equal(e1.partition(hosts[:10], 8),
                          np.repeat(np.arange(8), [2, 2] + [1] * 6))  # tiny lists: blocks


@pytest.mark.parametrize("kind", ["grid_ties", "dir800", "ba2k", "decimal_ties"])
def test_k32_buckets(kind, monkeypatch):
    """K = 32 buckets (variant 7: two 32-lane sub-groups per wave) bit-exact on
    the fixtures and on a tie-heavy grid of 3-decimal latencies."""
    monkeypatch.setenv("SHDR_VARIANT", "7")
    if kind == "decimal_ties":
        rng = np.random.default_rng(21)
        n = 60  # grid of 3-decimal latencies drawn from a small set: many exact ties
        vid = np.arange(n * n).reshape(n, n)
        ef = np.concatenate([vid[:, :-1].ravel(), vid[:-1, :].ravel(), vid.ravel()]).astype(np.int32)
        et = np.concatenate([vid[:, 1:].ravel(), vid[1:, :].ravel(), vid.ravel()]).astype(np.int32)
        lat = rng.choice([0.105, 0.215, 0.333, 1.005], len(ef))
        V = n * n
        og = po.OracleGraph(V, ef, et, lat, rng.uniform(0, 0.01, len(ef)), rng.uniform(0, 0.02, V))
        g = Graph.from_edges(V, ef, et, lat, og._keep[3], og._keep[4])
        src = rng.choice(V, 90, replace=False).astype(np.int32)
        dst = np.arange(0, V, 3, dtype=np.int32)
    else:
        z = load_sssp(kind)
        g = _graph_from_fixture(z)
        og = po.OracleGraph(int(z["V"]), z["efrom"], z["eto"], z["elat"], z["eloss"], z["vloss"], bool(z["directed"]))
        src, dst = z["sources"], z["targets"]
    t = Engine(g).compute(src, dst, hops=True)
    lat_o, rel_o, hops_o, rmin_o = og.routes(src, dst, po.MODE_CANONICAL, threads=8)
    assert np.array_equal(bits(t.lat), bits(lat_o)) and np.array_equal(bits(t.rel), bits(rel_o))
    assert np.array_equal(t.hops, hops_o) and np.array_equal(bits(t.row_min), bits(rmin_o))


@pytest.mark.parametrize("variant,mode,cl,kind,S", [
    ("4", "2", "2", "chunglu", 300), ("4", "1", "3", "chunglu", 300), ("6", "2", "4", "chunglu", 300),
    ("6", "1", "2", "chunglu", 1250), ("7", "1", "2", "chunglu", 300), ("7", "2", "3", "chunglu", 40),
    ("4", "2", "4", "chunglu", 3000), ("4", "1", "2", "dir800", 0), ("4", "2", "3", "grid_ties", 0),
    ("6", "2", "2", "ba2k", 0), ("4", "1", "3", "chunglu_all", 200), ("6", "2", "2", "chunglu_all", 200)])
def test_cluster_buckets(variant, mode, cl, kind, S, monkeypatch):
    """Cluster mode (SHDR_CLUSTER = cl workgroups per bucket, small shards):
    shared near-set planes, private far sets, cluster barriers, the split
    predecessor pass and epilogue — bit-exact against the oracle, K = 8/16/32,
    directed and tie-heavy graphs, fewer and more buckets than clusters, and
    again on the same engine. Pending mode 1 (far set in slot bytes) never runs
    clusters (routes.hip cluster_occupancy): those cases assert
    the plain layout was taken instead of the forced width, bit-exact."""
    monkeypatch.setenv("SHDR_VARIANT", variant)
    monkeypatch.setenv("SHDR_PENDING_LDS", mode)
    monkeypatch.setenv("SHDR_CLUSTER", cl)
    if kind.startswith("chunglu"):  # _all: every vertex a target (full predecessor pass)
        g = Graph.generate("chunglu", 12000, 3, 23)
        og = po.OracleGraph.from_graph(g)
        src = np.random.default_rng(S).choice(g.V, S, replace=False).astype(np.int32)
        dst = np.arange(0, g.V, 1 if kind == "chunglu_all" else 13, dtype=np.int32)
    else:
        z = load_sssp(kind)
        g = _graph_from_fixture(z)
        og = po.OracleGraph(int(z["V"]), z["efrom"], z["eto"], z["elat"], z["eloss"], z["vloss"], bool(z["directed"]))
        src, dst = z["sources"], z["targets"]
    eng = Engine(g)
    lat, rel, hops, rmin = og.routes(src, dst, po.MODE_CANONICAL, threads=8)
    for _ in range(2):
        t = eng.compute(src, dst, hops=True)
        lay = eng.last_layout()
        # the cluster kernel itself ran (no silent fallback to plain buckets);
        # PM 1 is gated off: the forced width must not be taken
        assert lay["cluster"] == (int(cl) if mode == "2" else 1) and lay["cluster_fallback"] == 0, lay
        assert lay["cluster_fallbacks_total"] == 0, lay
        assert np.array_equal(bits(t.lat), bits(lat)) and np.array_equal(bits(t.rel), bits(rel))
        assert np.array_equal(t.hops, hops) and np.array_equal(bits(t.row_min), bits(rmin))


@pytest.mark.parametrize("variant", ["4", "6"])
def test_pm1_cluster_round3_case(variant, monkeypatch):
    """The case that failed in round 3: Chung-Lu 7,000 vertices, 300
    sources, far set in slot bytes (PM 1), automatic layout. Round 3/4 picked 4-wide
    PM 1 clusters here; since round 5 PM 1 never runs clusters, so the product
    takes a plain layout (asserted) and every table of three fresh engines is
    bit-exact."""
    g = Graph.generate("chunglu", 7000, 3, 8)
    src = np.random.default_rng(4).choice(g.V, 300, replace=False).astype(np.int32)
    dst = np.arange(0, g.V, 11, dtype=np.int32)
    lat, rel, hops, rmin = po.OracleGraph.from_graph(g).routes(src, dst, po.MODE_CANONICAL, threads=8)
    monkeypatch.setenv("SHDR_PENDING_LDS", "1")
    monkeypatch.setenv("SHDR_VARIANT", variant)
    for _ in range(3):
        eng = Engine(g)
        t = eng.compute(src, dst, hops=True)
        lay = eng.last_layout()
        assert lay["cluster"] == 1 and lay["cluster_fallback"] == 0, lay
        assert np.array_equal(bits(t.lat), bits(lat)) and np.array_equal(bits(t.rel), bits(rel))
        assert np.array_equal(t.hops, hops) and np.array_equal(bits(t.row_min), bits(rmin))
        del eng


@pytest.mark.parametrize("S,want_cl", [(1250, 3), (2500, 3), (5000, 4), (6250, 1)])
def test_automatic_layout_wave_model(S, want_cl):
    """Default knobs: the wave model picks the cluster width from the shard size
    (256 CUs: 1,250 / 2,500 rows -> 3, 5,000 -> 4, 6,250 -> plain K=16 buckets
    with the partial group issued first); whatever it picks, sampled rows are
    bit-exact against the oracle and the row minima of every row against a
    plain-layout run."""
    g = Graph.generate("chunglu", 12000, 3, 29)
    og = po.OracleGraph.from_graph(g)
    src = np.random.default_rng(S).choice(g.V, S, replace=False).astype(np.int32)
    dst = np.arange(0, g.V, 13, dtype=np.int32)
    eng = Engine(g)
    t = eng.compute(src, dst, hops=True)
    lay = eng.last_layout()
    import torch
    if torch.cuda.get_device_properties(0).multi_processor_count == 256:
        assert lay["cluster"] == want_cl, lay
        if want_cl == 1:
            assert lay["partial_first"] == 1, lay
    rows = np.sort(np.random.default_rng(1).choice(S, 160, replace=False))
    lat, rel, hops, rmin = og.routes(src[rows], dst, po.MODE_CANONICAL, threads=8)
    assert np.array_equal(bits(t.lat[rows]), bits(lat)) and np.array_equal(bits(t.rel[rows]), bits(rel))
    assert np.array_equal(t.hops[rows], hops) and np.array_equal(bits(t.row_min[rows]), bits(rmin))
    os.environ["SHDR_CLUSTER"] = "1"
    try:
        plain = Engine(g).compute(src, dst, hops=True)
    finally:
        del os.environ["SHDR_CLUSTER"]
    assert np.array_equal(bits(t.lat), bits(plain.lat)) and np.array_equal(bits(t.rel), bits(plain.rel))
    assert np.array_equal(t.hops, plain.hops) and np.array_equal(bits(t.row_min), bits(plain.row_min))


def test_large_host_table_copy():
    """Host outputs of >= 256 MB per array (pre-faulted by worker threads while
    the kernels run, then copied): the table must equal the device-output table
    bit for bit."""
    import torch
    g = Graph.generate("chunglu", 20000, 3, 31)
    rng = np.random.default_rng(3)
    S = T = 6000  # 36e6 pairs: 288 MB per f64 array
    src = rng.choice(g.V, S, replace=False).astype(np.int32)
    dst = rng.choice(g.V, T, replace=False).astype(np.int32)
    eng = Engine(g)
    lat_d = torch.empty((S, T), dtype=torch.float64, device="cuda")
    rel_d = torch.empty((S, T), dtype=torch.float64, device="cuda")
    rmin_d = torch.empty((S,), dtype=torch.float64, device="cuda")
    eng.compute_device(src, dst, lat_d.data_ptr(), rel_d.data_ptr(), rmin_d.data_ptr(), None)
    torch.cuda.synchronize()
    t = eng.compute(src, dst)
    assert np.array_equal(bits(t.lat), bits(lat_d.cpu().numpy()))
    assert np.array_equal(bits(t.rel), bits(rel_d.cpu().numpy()))
    assert np.array_equal(bits(t.row_min), bits(rmin_d.cpu().numpy()))


@pytest.mark.parametrize("env", [{}, {"SHDR_CLUSTER": "2"}, {"SHDR_BALANCE": "1"}, {"SHDR_TAIL_MIN_WAVES": "1"},
                                 {"SHDR_CONCURRENT_TAIL": "0", "SHDR_TAIL_MIN_WAVES": "1"}])
def test_progressive_host_copy(env, monkeypatch):
    """Host outputs copied progressively (routes.hip: rows written in processing
    order, each finished bucket flags itself in host memory, the host copies
    finished rows through pinned staging and scatters them to the caller's rows
    while the launch runs), forced here on a small table with many small chunks:
    across layouts (plain + concurrent or serial half-width tail, cluster,
    balanced, a partial group issued first) the host table and row minima equal
    the device-output table bit for bit."""
    import torch
    monkeypatch.setenv("SHDR_PROGRESSIVE_MIN_MB", "0.001")
    monkeypatch.setenv("SHDR_PROGRESSIVE_CHUNK_MB", "0.2")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = Graph.generate("chunglu", 20000, 3, 37)
    rng = np.random.default_rng(9)
    src = rng.choice(g.V, 6003, replace=False).astype(np.int32)
    dst = rng.choice(g.V, 2500, replace=False).astype(np.int32)
    eng = Engine(g)
    t = eng.compute(src, dst)
    lay = eng.last_layout()
    assert lay["progressive"] == 1, lay
    S, T = len(src), len(dst)
    lat_d = torch.empty((S, T), dtype=torch.float64, device="cuda")
    rel_d = torch.empty((S, T), dtype=torch.float64, device="cuda")
    rmin_d = torch.empty((S,), dtype=torch.float64, device="cuda")
    eng.compute_device(src, dst, lat_d.data_ptr(), rel_d.data_ptr(), rmin_d.data_ptr(), None)
    torch.cuda.synchronize()
    assert eng.last_layout()["progressive"] == 0
    assert np.array_equal(bits(t.lat), bits(lat_d.cpu().numpy()))
    assert np.array_equal(bits(t.rel), bits(rel_d.cpu().numpy()))
    assert np.array_equal(bits(t.row_min), bits(rmin_d.cpu().numpy()))
    rows = np.sort(rng.choice(S, 12, replace=False))
    og = po.OracleGraph.from_graph(g)
    lat, rel, _, rmin = og.routes(src[rows], dst, po.MODE_CANONICAL, threads=8)
    assert np.array_equal(bits(t.lat[rows]), bits(lat)) and np.array_equal(bits(t.rel[rows]), bits(rel))


@pytest.mark.gpu
def test_progressive_staging_grows_with_T(monkeypatch):
    """One engine, two progressive host-output computes whose second T needs a
    larger pinned staging buffer (0.2 MB chunks: T = 2,500 stages 2 x 10 rows of
    20,000 B, T = 2,600 stages 2 x 10 rows of 20,800 B): the staging buffer grows
    instead of being overrun, and both tables equal their device-output tables."""
    import torch
    monkeypatch.setenv("SHDR_PROGRESSIVE_MIN_MB", "0.001")
    monkeypatch.setenv("SHDR_PROGRESSIVE_CHUNK_MB", "0.2")
    g = Graph.generate("chunglu", 20000, 3, 37)
    rng = np.random.default_rng(11)
    src = rng.choice(g.V, 3001, replace=False).astype(np.int32)
    eng = Engine(g)
    for T in (2500, 2600):
        dst = rng.choice(g.V, T, replace=False).astype(np.int32)
        t = eng.compute(src, dst)
        assert eng.last_layout()["progressive"] == 1
        lat_d = torch.empty((len(src), T), dtype=torch.float64, device="cuda")
        rel_d = torch.empty((len(src), T), dtype=torch.float64, device="cuda")
        eng.compute_device(src, dst, lat_d.data_ptr(), rel_d.data_ptr(), None, None)
        torch.cuda.synchronize()
        assert np.array_equal(bits(t.lat), bits(lat_d.cpu().numpy()))
        assert np.array_equal(bits(t.rel), bits(rel_d.cpu().numpy()))
