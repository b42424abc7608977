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
