import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
from oracle import py_oracle as po
from shadow_amd.routes import Engine, Graph
from tests.util import load_sssp, bits
for kind in ["dir800", "ba2k", "grid_ties"]:
    z = load_sssp(kind)
    V = int(z["V"])
    g = Graph.from_edges(V, z["efrom"], z["eto"], z["elat"], z["eloss"], z["vloss"], directed=bool(z["directed"]))
    rng = np.random.default_rng(7)
    dst = np.sort(rng.choice(V, size=max(1, V // 5), replace=False)).astype(np.int32)
    src = z["sources"]
    eng = Engine(g)
    t = eng.compute(src, dst, hops=True)
    full = eng.compute(src, np.arange(V, dtype=np.int32), hops=True)
    bad = bits(t.lat) != bits(full.lat[:, dst])
    print(kind, "S", len(src), "T", len(dst), "mismatch", bad.sum(), "nan in chain", np.isnan(t.lat).sum(), "nan in full", np.isnan(full.lat[:, dst]).sum())
    ii, jj = np.nonzero(bad)
    for i, j in list(zip(ii, jj))[:5]:
        print("  ", i, j, src[i], dst[j], t.lat[i, j], full.lat[i, dst[j]], t.hops[i, j], full.hops[i, dst[j]])
