"""Host graph: GraphML reader (igraph indexing), validation, canonical edges,
generators. Cross-checked against an independent xml.etree reader."""
import lzma
import os
import xml.etree.ElementTree as ET

import numpy as np
import pytest

from shadow_amd.routes import Graph

NS = "{http://graphml.graphdrawing.org/xmlns}"


def etree_read(text):
    root = ET.fromstring(text)
    keys = {k.get("id"): k.get("attr.name") for k in root.iter(NS + "key")}
    graph = root.find(NS + "graph")
    idx, ids, ef, et, lat, vloss = {}, [], [], [], [], {}

    def vid(x):
        if x not in idx:
            idx[x] = len(ids)
            ids.append(x)
        return idx[x]

    for el in graph:
        if el.tag == NS + "node":
            v = vid(el.get("id"))
            for d in el.findall(NS + "data"):
                if keys[d.get("key")] == "packetloss":
                    vloss[v] = float(d.text)
        elif el.tag == NS + "edge":
            ef.append(vid(el.get("source")))
            et.append(vid(el.get("target")))
            for d in el.findall(NS + "data"):
                if keys[d.get("key")] == "latency":
                    lat.append(float(d.text))
    return ids, ef, et, lat, vloss


@pytest.mark.parametrize("name", ["simple", "full", "plab"])
def test_graphml_reader_matches_etree(name, topo_paths):
    text = open(topo_paths[name]).read()
    ids, ef, et, lat, vloss = etree_read(text)
    g = Graph.load_graphml(topo_paths[name])
    assert g.V == len(ids) and g.E == len(ef)
    assert [g.vertex_str("id", v) for v in range(g.V)] == ids
    gef, get, glat, glo, gvl = g.export()
    assert np.array_equal(gef, ef) and np.array_equal(get, et)
    assert np.array_equal(glat, np.array(lat))
    for v, p in vloss.items():
        assert gvl[v] == p
    info = g.check()
    assert info.is_connected and info.cluster_count == 1 and info.is_complete and not info.is_directed
    assert info.bad_latency_edges == 0 and info.self_loops == g.V
    # string + numeric vertex attributes as igraph's cattribute table keeps them
    assert g.vertex_str("type", 0) != "" and g.vertex_num("bandwidthup", 0) > 0


def test_forward_referenced_nodes_get_first_appearance_index():
    text = """<graphml xmlns="http://graphml.graphdrawing.org/xmlns">
      <key attr.name="latency" attr.type="double" for="edge" id="d7"/>
      <key attr.name="packetloss" attr.type="double" for="node" id="d0"><default>0.5</default></key>
      <graph edgedefault="undirected">
        <node id="a"/>
        <edge source="a" target="c"><data key="d7">2.0</data></edge>
        <node id="b"><data key="d0">0.25</data></node>
        <node id="c"/>
        <edge source="b" target="c"><data key="d7"> 3.5 </data></edge>
      </graph></graphml>"""
    g = Graph.parse_graphml(text)
    assert [g.vertex_str("id", v) for v in range(3)] == ["a", "c", "b"]
    assert g.vertex_num("packetloss", 0) == 0.5  # <default>
    assert g.vertex_num("packetloss", 2) == 0.25
    assert g.edge_num("latency", 1) == 3.5
    assert np.isnan(g.edge_num("packetloss", 0))  # undeclared key -> NaN
    info = g.check()
    assert info.is_connected and not info.is_complete


def test_entities_comments_cdata():
    text = """<?xml version="1.0"?><!-- c --><graphml xmlns="http://graphml.graphdrawing.org/xmlns">
      <key attr.name="type" attr.type="string" for="node" id="t"/>
      <key attr.name="latency" attr.type="double" for="edge" id="l"/>
      <graph edgedefault="directed"><node id="x&amp;y"><data key="t"><![CDATA[a<b&c]]></data></node>
      <node id="z"><data key="t">q&lt;r</data></node>
      <edge source="x&amp;y" target="z"><data key="l">1</data></edge>
      <edge source="z" target="x&amp;y"><data key="l">1</data></edge></graph></graphml>"""
    g = Graph.parse_graphml(text)
    assert g.directed and g.V == 2
    assert g.vertex_str("id", 0) == "x&y"
    assert g.vertex_str("type", 0) == "a<b&c" and g.vertex_str("type", 1) == "q<r"
    assert g.check().is_connected


def test_connectivity_and_completeness_rules():
    # two components -> not connected (topology_new rejects it, :255-258)
    g = Graph.from_edges(4, [0, 2], [1, 3], [1.0, 1.0])
    info = g.check()
    assert not info.is_connected and info.cluster_count == 2
    # directed: 0->1 only -> not strongly connected
    g = Graph.from_edges(2, [0], [1], [1.0], directed=True)
    info = g.check()
    assert not info.is_connected and info.cluster_count == 2
    # undirected triangle without self-loops: incident count 2 < V=3 -> incomplete
    g = Graph.from_edges(3, [0, 1, 2], [1, 2, 0], [1.0] * 3)
    assert not g.check().is_complete
    # with self-loops: 2 + 2 - 1 = 3 >= 3 -> complete (:187-201)
    g = Graph.from_edges(3, [0, 1, 2, 0, 1, 2], [1, 2, 0, 0, 1, 2], [1.0] * 6)
    assert g.check().is_complete
    # directed complete needs out-degree >= V including the self-loop
    ef = [a for a in range(3) for b in range(3)]
    et = [b for a in range(3) for b in range(3)]
    g = Graph.from_edges(3, ef, et, [1.0] * 9, directed=True)
    assert g.check().is_complete
    # latency <= 0 is counted (the reference error()s, :414-419)
    g = Graph.from_edges(2, [0, 0], [1, 1], [0.0, -1.0])
    assert g.check().bad_latency_edges == 2


def test_canonical_edge_is_lowest_index():
    g = Graph.from_edges(3, [1, 0, 1, 2], [0, 1, 2, 2], [5.0, 6.0, 7.0, 8.0])
    assert g.get_eid(0, 1) == 0 and g.get_eid(1, 0) == 0  # undirected: either orientation
    assert g.get_eid(2, 2) == 3 and g.get_eid(0, 2) == -1
    d = Graph.from_edges(2, [1, 0], [0, 1], [5.0, 6.0], directed=True)
    assert d.get_eid(0, 1) == 1 and d.get_eid(1, 0) == 0


@pytest.mark.parametrize("kind,n,m", [("ba", 5000, 3), ("chunglu", 20000, 3)])
def test_generators(kind, n, m):
    g1 = Graph.generate(kind, n, m, 7)
    g2 = Graph.generate(kind, n, m, 7)
    a, b = g1.export(), g2.export()
    for x, y in zip(a, b):
        assert np.array_equal(x, y)  # deterministic
    ef, et, lat, lo, vl = a
    loops = ef == et
    assert loops.sum() == n  # one self-loop per vertex
    assert ((lat[~loops] >= 1) & (lat[~loops] <= 100)).all()
    assert ((lat[loops] >= 0.5) & (lat[loops] <= 5)).all()
    assert ((lo >= 0) & (lo <= 0.01)).all() and ((vl >= 0) & (vl <= 0.02)).all()
    key = np.minimum(ef, et).astype(np.int64) * n + np.maximum(ef, et)
    assert len(np.unique(key)) == len(key)  # simple graph
    info = g1.check()
    assert info.is_connected and not info.is_complete
    mean_deg = 2 * (~loops).sum() / n
    assert 5.0 < mean_deg < 7.0


def _same_graph(a, b):
    assert (a.V, a.E, a.directed) == (b.V, b.E, b.directed)
    for x, y in zip(a.export(), b.export()):
        assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))
    for v in range(0, a.V, max(1, a.V // 50)):
        for attr in ("id", "ip", "geocode", "type"):
            assert a.vertex_str(attr, v) == b.vertex_str(attr, v)
        assert a.vertex_num("bandwidthup", v) == b.vertex_num("bandwidthup", v) or np.isnan(a.vertex_num("bandwidthup", v))


@pytest.mark.parametrize("name", ["simple", "full", "plab"])
def test_binary_image_round_trip(name, topo_paths, tmp_path):
    g = Graph.load_graphml(topo_paths[name])
    p = tmp_path / f"{name}.shdrgraph"
    g.save_binary(str(p))
    _same_graph(g, Graph.load_binary(str(p)))


def test_graphml_cache(topo_paths, tmp_path, monkeypatch):
    """SHDR_GRAPH_CACHE: the first load writes a content-keyed image, later loads
    (of any file with the same bytes) read it back; a corrupt image is ignored."""
    import glob
    import shutil
    monkeypatch.setenv("SHDR_GRAPH_CACHE", str(tmp_path))
    g1 = Graph.load_graphml(topo_paths["full"])
    imgs = glob.glob(str(tmp_path / "*.shdrgraph"))
    assert len(imgs) == 1
    copy = tmp_path / "renamed.graphml.xml"
    shutil.copyfile(topo_paths["full"], copy)
    _same_graph(g1, Graph.load_graphml(str(copy)))
    open(imgs[0], "wb").write(b"SHDRGRF1garbage")
    _same_graph(g1, Graph.load_graphml(topo_paths["full"]))
    with pytest.raises(Exception):
        Graph.load_binary(str(tmp_path / "missing.shdrgraph"))


@pytest.mark.parametrize("src", ["simple", "full", "plab", "chunglu", "directed"])
def test_graphml_writer_round_trip(src, topo_paths, tmp_path):
    """shdr_graph_save_graphml is lossless: reading the file back gives the same
    vertex/edge order, endpoints and every attribute bit for bit."""
    if src in topo_paths:
        g = Graph.load_graphml(topo_paths[src])
    elif src == "chunglu":
        g = Graph.generate("chunglu", 20000, 3, 3)
    else:
        rng = np.random.default_rng(1)
        g = Graph.from_edges(50, rng.integers(0, 50, 300), rng.integers(0, 50, 300), rng.uniform(1, 9, 300),
                             rng.uniform(0, 0.1, 300), rng.uniform(0, 0.1, 50), directed=True)
    p = tmp_path / "out.graphml.xml"
    g.save_graphml(str(p))
    _same_graph(g, Graph.load_graphml(str(p)))


def test_generated_vertices_have_distinct_ips():
    g = Graph.generate("ba", 70000, 2, 1)
    ips = {g.vertex_str("ip", v) for v in range(0, g.V)}
    assert len(ips) == g.V and g.vertex_str("ip", 65536 + 258) == "10.1.1.2"


def _image(g, path):
    g.save_binary(path)
    with open(path, "rb") as f:
        return f.read()


_HDR = ('<?xml version="1.0"?>\n<graphml xmlns="http://graphml.graphdrawing.org/xmlns">\n'
        '<key id="d0" for="node" attr.name="packetloss" attr.type="double"><default>0.25</default></key>\n'
        '<key id="d1" for="node" attr.name="type" attr.type="string"><default>net</default></key>\n'
        '<key id="d2" for="edge" attr.name="latency" attr.type="double"/>\n'
        '<key id="d3" for="edge" attr.name="up" attr.type="boolean"/>\n'
        '<key id="d4" for="all" attr.name="note" attr.type="string"/>\n'
        '<graph edgedefault="undirected">\n')
_BODIES = {
    # edge endpoints before their <node>, duplicate node (last value wins), defaults,
    # self-closing and empty <data>, entities in ids and values, unknown keys,
    # <data> outside any element, boolean values, a <desc> child
    "plain": ('<edge source="x&amp;1" target="b"><data key="d2">2.5</data><data key="d3"> True </data></edge>\n'
              '<node id="b"><data key="d0">0.125</data><desc>kept out</desc></node>\n'
              '<node id="x&amp;1"><data key="d1">a&lt;b</data><data key="d9">7</data></node>\n'
              '<node id="b"><data key="d0">0.5</data><data key="d4"></data></node>\n'
              '<data key="d0">9</data>\n'
              '<node id="c"/>\n<edge source="c" target="b"><data key="d2"/></edge>\n'
              '<edge source="b" target="b"><data key="d2">1e-3</data><data key="d4">n</data></edge>\n'),
    # constructs the parallel reader hands back to the serial one
    "comment": '<node id="a"/><!-- c --><node id="b"/><edge source="a" target="b"><data key="d2">1</data></edge>\n',
    "cdata": '<node id="a"><data key="d1"><![CDATA[x&y]]></data></node><node id="b"/>'
             '<edge source="a" target="b"><data key="d2">1</data></edge>\n',
    "nested": '<node id="a"><graph id="s"><node id="q"/></graph></node><node id="b"/>'
              '<edge source="a" target="b"><data key="d2">1</data></edge>\n',
}


@pytest.mark.parametrize("body", sorted(_BODIES))
def test_parallel_graphml_reader_identical(body, tmp_path, monkeypatch):
    """The multi-threaded reader (documents >= 8 MB by default) gives the same
    graph, byte for byte in the binary image, as the serial reader, on the
    corner cases of igraph's conventions and on the constructs it hands back."""
    doc = _HDR + _BODIES[body] + "</graph>\n</graphml>\n"
    imgs = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("SHDR_GRAPHML_PARALLEL", mode)
        imgs[mode] = _image(Graph.parse_graphml(doc), str(tmp_path / f"g{mode}.bin"))
    assert imgs["0"] == imgs["1"]


def test_parallel_graphml_reader_large(tmp_path, monkeypatch, topo_paths):
    """A generated 20k-vertex topology written as GraphML and the bundled files:
    serial and parallel readers agree byte for byte."""
    g = Graph.generate("chunglu", 20000, 3, 5)
    path = str(tmp_path / "g.graphml")
    g.save_graphml(path)
    for p in [path] + [topo_paths[n] for n in ("full", "plab")]:
        imgs = {}
        for mode in ("0", "1"):
            monkeypatch.setenv("SHDR_GRAPHML_PARALLEL", mode)
            imgs[mode] = _image(Graph.load_graphml(p), str(tmp_path / f"i{mode}.bin"))
        assert imgs["0"] == imgs["1"], p


def test_graphml_writer_fallback_ids_do_not_collide(tmp_path):
    """A vertex without an id is written as "n<v>", made unique against the ids
    the graph already has (else reading the file back would merge two vertices);
    a name held both as a numeric and as a string column is refused."""
    doc = b'''<?xml version="1.0"?><graphml xmlns="http://graphml.graphdrawing.org/xmlns">
<key id="k0" for="edge" attr.name="latency" attr.type="double"/>
<graph edgedefault="undirected">
<node id=""/><node id="n0"/><node id="n0_"/><node id="n1"/>
<edge source="" target="n0"><data key="k0">2.5</data></edge>
<edge source="n0" target="n1"><data key="k0">1.5</data></edge>
<edge source="n0_" target="n1"><data key="k0">4.0</data></edge>
</graph></graphml>'''
    g = Graph.parse_graphml(doc)
    assert g.V == 4 and g.vertex_str("id", 0) == ""
    p = tmp_path / "ids.graphml"
    g.save_graphml(str(p))
    h = Graph.load_graphml(str(p))
    ids = [h.vertex_str("id", v) for v in range(h.V)]
    assert h.V == 4 and len(set(ids)) == 4 and ids[1:] == ["n0", "n0_", "n1"], ids
    assert h.E == g.E
    for e in range(g.E):
        assert h.edge_num("latency", e) == g.edge_num("latency", e)
    both = b'''<?xml version="1.0"?><graphml xmlns="http://graphml.graphdrawing.org/xmlns">
<key id="a" for="node" attr.name="x" attr.type="double"/><key id="b" for="node" attr.name="x" attr.type="string"/>
<key id="k0" for="edge" attr.name="latency" attr.type="double"/>
<graph edgedefault="undirected"><node id="u"><data key="a">1</data></node><node id="v"><data key="b">s</data></node>
<edge source="u" target="v"><data key="k0">1.0</data></edge></graph></graphml>'''
    g2 = Graph.parse_graphml(both)
    import pytest as _pt
    from shadow_amd.routes import ShdrError
    with _pt.raises(ShdrError):
        g2.save_graphml(str(tmp_path / "both.graphml"))
