#!/usr/bin/env python3
"""Padding share of the relaxation's work items (CPU only; DESIGN.md §3.1, half-block pairs).

A vertex's arcs are packed 8 to a 128-B block, its last block padded. For the
expandable vertices of a workload (degree > 1, the pendant rule approximated by
degree), print the item slots that carry no arc: one item per block, then with
last blocks of <= 4 arcs relaxed two to an item (half-block pairs), then, for
comparison, with last blocks of <= 2 arcs four to an item. Unweighted by how often
a vertex is expanded.   usage: python tools/pad_share.py [cfg5|cfg4]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402

g, _, _, _ = bench.make_workload(sys.argv[1] if len(sys.argv) > 1 else "cfg5")
ef, et, _, _, _ = g.export()
m = ef != et
deg = np.bincount(np.concatenate([ef[m], et[m]]), minlength=g.V)
d = deg[deg > 1]
blocks = (d + 7) // 8
last = d - (blocks - 1) * 8
arcs = d.sum()
plain = blocks.sum()
pairs = (blocks - 1).sum() + (last > 4).sum() + (last <= 4).sum() / 2
quads = (blocks - 1).sum() + (last > 4).sum() + ((last > 2) & (last <= 4)).sum() / 2 + (last <= 2).sum() / 4
print(f"expandable vertices {len(d)}, arcs {arcs}")
for name, items in (("one item per block", plain), ("half-block pairs", pairs), ("quarter groups", quads)):
    print(f"{name:20s} items {items:12.0f}  padding share {1 - arcs / (8 * items):.3f}")
print("degree histogram (2..19, >=20):", np.bincount(np.minimum(d, 20))[2:].tolist())
