"""Host -> vertex attachment of the drop-in (topology_attach)
against the restated reference algorithm (oracle/attach.py), on the bundled
topologies: hint filtering by type / geocode, exact-IP matches, longest-prefix
matching, and the rand_r-driven uniform pick of each host's Random.

Runs on CPU: attaching never touches the GPU.
"""
import lzma
import os
import xml.etree.ElementTree as ET

import numpy as np
import pytest

from oracle import attach as oa
from shadow_amd import topology as top

NS = "{http://graphml.graphdrawing.org/xmlns}"


def vertex_attrs(path):
    """Vertex string attributes in igraph index order (independent xml.etree reader)."""
    root = ET.parse(path).getroot()
    keys = {k.get("id"): k.get("attr.name") for k in root.iter(NS + "key") if k.get("for") == "node"}
    out, index = [], {}
    for el in root.find(NS + "graph"):
        if el.tag == NS + "node":
            d = {"id": el.get("id")}
            for dd in el.findall(NS + "data"):
                if dd.get("key") in keys:
                    d[keys[dd.get("key")]] = dd.text or ""
            index[el.get("id")] = len(out)
            out.append(d)
    return out


SCENARIOS = [
    # (ip hint, geocode hint, type hint)
    (None, None, None),
    (None, None, "cluster"),
    (None, None, "relay"),          # no vertex of that type: falls back to all
    (None, "SD", None),
    (None, "sd", "CLUSTER"),        # case-insensitive (g_ascii_strcasecmp)
    (None, "XX", "cluster"),        # geocode misses, type hits
    ("190.181.151.39", None, None),  # exact IP match
    ("190.181.0.1", None, None),     # longest-prefix match among usable IPs
    ("190.181.0.1", "SD", None),     # prefix hint, but the filtered set has no usable IP
    ("10.0.0.1", None, "cluster"),
    ("not-an-ip", None, None),
]


@pytest.mark.parametrize("name", ["full", "plab", "simple"])
def test_attach_matches_reference_algorithm(name, topo_paths):
    verts = vertex_attrs(topo_paths[name])
    t = top.Topology.new(topo_paths[name])
    assert t is not None
    n = 0
    for si, (iph, geo, typ) in enumerate(SCENARIOS):
        for k in range(25):
            seed = 1000 * si + k
            addr = top.Address(f"11.{si}.{k // 250}.{k % 250 + 1}", f"h{si}-{k}")
            want = oa.find_vertex(verts, oa.Random(seed), iph, geo, typ)
            bw_down, bw_up = t.attach(addr, top.Random(seed), iph, geo, typ)
            got = t.vertex_of(addr)
            assert got == want, (name, iph, geo, typ, seed, got, want)
            if want >= 0 and "bandwidthdown" in verts[want]:
                assert bw_down == int(float(verts[want]["bandwidthdown"]))
                assert bw_up == int(float(verts[want]["bandwidthup"]))
            n += 1
    assert n == 25 * len(SCENARIOS)
    t.free()


def test_random_stream_is_libc_rand_r():
    """The drop-in's Random (shim, = shd-random.c) and the oracle's draw the same values."""
    a, b = top.Random(7), oa.Random(7)
    xs = [a.next_double() for _ in range(100)]
    ys = [b.next_double() for _ in range(100)]
    assert xs == ys
    assert all(0.0 <= x <= 1.0 for x in xs)


def test_reattach_replaces_mapping(topo_paths):
    t = top.Topology.new(topo_paths["full"])
    a = top.Address("11.0.0.1")
    t.attach(a, top.Random(1), "190.181.151.39")
    v1 = t.vertex_of(a)
    t.attach(a, top.Random(2), None, "SD")
    v2 = t.vertex_of(a)
    verts = vertex_attrs(topo_paths["full"])
    assert verts[v1]["ip"] == "190.181.151.39"
    assert verts[v2]["geocode"] == "SD"
    t.detach(a)
    assert t.vertex_of(a) == -1
    t.free()


def test_attach_index_on_synthetic_attributes(tmp_path):
    """Duplicate IPs (several exact matches), mixed-case types and geocodes, many
    unusable IPs: the indexed candidate sets must pick what the scan picks."""
    from tests.util import write_graphml
    rng = np.random.default_rng(3)
    V = 600
    ef = np.arange(1, V, dtype=np.int32)
    et = rng.integers(0, np.arange(1, V)).astype(np.int32)
    ips = [rng.choice(["0.0.0.0", f"10.{i % 7}.{i % 3}.1", f"172.16.{i % 5}.{i % 11}"]) for i in range(V)]
    types = [rng.choice(["relay", "Relay", "client", "EXIT"]) for _ in range(V)]
    geos = [rng.choice(["US", "us", "DE", "FR", "cn"]) for _ in range(V)]
    p = tmp_path / "attrs.graphml.xml"
    write_graphml(p, V, ef, et, np.full(V - 1, 5.0), np.zeros(V - 1), np.zeros(V), ips=ips, types=types, geocodes=geos)
    verts = vertex_attrs(str(p))
    t = top.Topology.new(str(p))
    hints = [(None, None, None), (None, "US", "relay"), (None, "de", None), (None, None, "exit"),
             ("10.3.0.1", None, None), ("10.3.0.1", "FR", "client"), ("172.16.2.9", "cn", None),
             ("172.16.0.0", None, "RELAY"), ("8.8.8.8", "us", "client")]
    for si, (iph, geo, typ) in enumerate(hints):
        for k in range(40):
            seed = 77 * si + k
            addr = top.Address(f"11.{si}.0.{k + 1}")
            want = oa.find_vertex(verts, oa.Random(seed), iph, geo, typ)
            t.attach(addr, top.Random(seed), iph, geo, typ)
            assert t.vertex_of(addr) == want, (iph, geo, typ, seed)
    t.free()
