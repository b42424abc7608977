#!/usr/bin/env python3
"""Cluster-mode parity repro (experiments only): one partition shard, several
SHDR_CLUSTER settings, each run twice, compared with the oracle."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from oracle import py_oracle as po  # noqa: E402
from shadow_amd.routes import Engine, Graph  # noqa: E402


def bits(x):
    return np.ascontiguousarray(x).view(np.uint64)


g = Graph.generate("chunglu", int(os.environ.get("N", "20000")), 3, 2)
hosts = np.sort(np.random.default_rng(3).choice(g.V, 3001, replace=False)).astype(np.int32)
part = Engine(g).partition(hosts, 8)
dst = hosts[::7] if os.environ.get("ALLDST") != "1" else np.arange(g.V, dtype=np.int32)
src = hosts[part == 0] if os.environ.get("FULL") != "1" else hosts
og = po.OracleGraph.from_graph(g)
lat, rel, hops, rmin = og.routes(src, dst, po.MODE_CANONICAL, threads=16)
for conf in sys.argv[1:]:
    env = dict(kv.split("=") for kv in conf.split())
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    eng = Engine(g)
    for rep in range(3):
        t = eng.compute(src, dst, hops=True)
        bad_r = bits(t.rel) != bits(rel)
        bad_h = t.hops != hops
        bad_l = bits(t.lat) != bits(lat)
        rows = np.unique(np.nonzero(bad_r)[0])
        print(f"[{conf}] rep {rep}: lat bad {bad_l.sum()} rel bad {bad_r.sum()} hops bad {bad_h.sum()} rows {rows[:12].tolist()}"
              f" cols {np.unique(np.nonzero(bad_r)[1])[:12].tolist()}", flush=True)
        if bad_l.any():
            d = (t.lat - lat)[bad_l]
            print("   lat diff: gpu>oracle", int((d > 0).sum()), "gpu<oracle", int((d < 0).sum()), "max", float(np.abs(d).max()), flush=True)
        if bad_h.any():
            i, j = np.argwhere(bad_h)[0]
            print("   first: src", src[i], "dst", dst[j], "hops gpu", t.hops[i, j], "oracle", hops[i, j], flush=True)
    del eng
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
