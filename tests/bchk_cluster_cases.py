"""Cluster-mode cases run once each through the bounds-checked flavour
(libshdtopology_bchk.so, built with -DSHDR_BCHK by `make -C shadow_amd bchk`).

Started by tests/test_gpu_bchk.py in a fresh process with SHDR_LIB_VARIANT=bchk
(one library per process). The flavour clamps out-of-range slot, arc and work-list
indices and flags them in the device guard word (codes >= 256), and poisons every
predecessor entry at bucket start so a walk that reaches an entry the
predecessor pass never wrote trips guard 32: a lost chain-pass mark (the
round-2 race, commit 1d88a84) fails deterministically here instead of showing as
a wrong path under some timings. A tripped guard makes shdr_routes_compute fail,
which raises. Every table must also equal the oracle's canonical mode bit for bit.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from oracle import py_oracle as po  # noqa: E402
from shadow_amd import _lib  # noqa: E402
from shadow_amd.routes import Engine, Graph, lib_kernel_sha, src_kernel_sha  # noqa: E402
from tests.util import bits, load_sssp  # noqa: E402

# (variant, pending mode, cluster width, graph, sources): the cases of
# test_gpu_parity.py::test_cluster_buckets
CASES = [
    ("4", "2", "2", "chunglu", 300), ("4", "1", "3", "chunglu", 300), ("6", "2", "4", "chunglu", 300),
    ("6", "1", "2", "chunglu", 1250), ("7", "1", "2", "chunglu", 300), ("7", "2", "3", "chunglu", 40),
    ("4", "2", "4", "chunglu", 3000), ("4", "1", "2", "dir800", 0), ("4", "2", "3", "grid_ties", 0),
    ("6", "2", "2", "ba2k", 0), ("4", "1", "3", "chunglu_all", 200), ("6", "2", "2", "chunglu_all", 200)]


def main() -> int:
    assert _lib.LIB_PATH.endswith("libshdtopology_bchk.so"), _lib.LIB_PATH
    # the flavour was built from the tree's sources (tests/conftest.py rebuilds stale flavours)
    assert lib_kernel_sha() == src_kernel_sha(), (lib_kernel_sha(), src_kernel_sha())
    cl_graph = Graph.generate("chunglu", 12000, 3, 23)
    cl_oracle = po.OracleGraph.from_graph(cl_graph)
    for variant, mode, cl, kind, S in CASES:
        os.environ["SHDR_VARIANT"] = variant
        os.environ["SHDR_PENDING_LDS"] = mode
        os.environ["SHDR_CLUSTER"] = cl
        if kind.startswith("chunglu"):
            g, og = cl_graph, cl_oracle
            src = np.random.default_rng(S).choice(g.V, S, replace=False).astype(np.int32)
            dst = np.arange(0, g.V, 1 if kind == "chunglu_all" else 13, dtype=np.int32)
        else:
            z = load_sssp(kind)
            g = Graph.from_edges(int(z["V"]), z["efrom"], z["eto"], z["elat"], z["eloss"], z["vloss"],
                                 directed=bool(z["directed"]))
            og = po.OracleGraph(int(z["V"]), z["efrom"], z["eto"], z["elat"], z["eloss"], z["vloss"],
                                bool(z["directed"]))
            src, dst = z["sources"], z["targets"]
        eng = Engine(g)
        t = eng.compute(src, dst, hops=True)  # raises on a tripped guard
        lay = eng.last_layout()
        # pending mode 1 never runs clusters (routes.hip cluster_occupancy): plain layout
        assert lay["cluster"] == (int(cl) if mode == "2" else 1) and lay["cluster_fallback"] == 0, (kind, lay)
        lat, rel, hops, rmin = og.routes(src, dst, po.MODE_CANONICAL, threads=8)
        ok = (np.array_equal(bits(t.lat), bits(lat)) and np.array_equal(bits(t.rel), bits(rel))
              and np.array_equal(t.hops, hops) and np.array_equal(bits(t.row_min), bits(rmin)))
        assert ok, (variant, mode, cl, kind, S)
        print(f"bchk ok: variant {variant} mode {mode} cl {cl} {kind} S={len(src)}", flush=True)
        del eng
    print(f"bchk cluster cases: {len(CASES)} passed", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
