#!/usr/bin/env python3
"""Wide parity sweep at a BASELINE config (evidence, not a test): the whole S x T
table on the GPU exactly as bench.py builds it, then ROWS seeded rows (half of
them from the concurrent tail launch when it ran) against the oracle's canonical
mode and its restated igraph mode, bit for bit (lat, rel, hops, row minimum).
tests/test_gpu_parity.py::test_baseline_workload_full_table does the same on 32 /
64 rows inside the suite; this widens it to hundreds.

usage: python tools/parity_sweep.py [cfg5|cfg4] [ROWS=256] [SEED=4242]
PART=N: every part of Engine.partition(hosts, N) in turn (the strong-scaling shards,
whose layout may be cluster mode), ROWS rows sampled per part."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from oracle import py_oracle as po  # noqa: E402
from shadow_amd.routes import Engine  # noqa: E402


def bits(a):
    return np.ascontiguousarray(a).view(np.uint64 if a.dtype == np.float64 else a.dtype)


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "cfg5"
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 4242
    g, hosts, _, _ = bench.make_workload(wl)
    nparts = int(os.environ.get("PART", "0"))
    if nparts:
        part = Engine(g).partition(hosts, nparts)
        return max(sweep(wl, g, hosts[part == p], hosts, rows, seed, f"part {p}/{nparts}") for p in range(nparts))
    return sweep(wl, g, hosts, hosts, rows, seed, "whole table")


def sweep(wl, g, src, hosts, rows, seed, label):
    S, T = len(src), len(hosts)
    dev = torch.device("cuda", 0)
    lat = torch.empty((S, T), dtype=torch.float64, device=dev)
    rel = torch.empty_like(lat)
    hops = torch.empty((S, T), dtype=torch.int32, device=dev)
    rmin = torch.empty((S,), dtype=torch.float64, device=dev)
    eng = Engine(g)
    t0 = time.perf_counter()
    eng.compute_device(src, hosts, lat.data_ptr(), rel.data_ptr(), rmin.data_ptr(), hops.data_ptr(),
                       stream=torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    gpu_s = time.perf_counter() - t0
    lay = eng.last_layout()
    order = eng.row_order()
    main_rows, tail_rows = order[:lay["rows_main"]], order[lay["rows_main"]:]
    rng = np.random.default_rng(seed)
    rows = min(rows, S)
    k_tail = min(len(tail_rows), rows // 2)
    pick = np.unique(np.concatenate([rng.choice(main_rows, min(len(main_rows), rows - k_tail), replace=False),
                                     rng.choice(tail_rows, k_tail, replace=False) if k_tail else
                                     np.empty(0, np.int32)]))
    og = po.OracleGraph.from_graph(g)
    threads = min(16, len(os.sched_getaffinity(0)))
    idx = torch.as_tensor(pick, device=dev)
    glat, grel = lat[idx].cpu().numpy(), rel[idx].cpu().numpy()
    ghops, grmin = hops[idx].cpu().numpy(), rmin[idx].cpu().numpy()
    out = {"workload": wl, "shard": label, "S": S, "rows": int(len(pick)), "tail_rows": int(sum(int(p) in set(tail_rows.tolist()) for p in pick)),
           "seed": seed, "layout": lay, "gpu_table_s": round(gpu_s, 3), "kernel_sha": bench.kernel_sha()}
    for mode, name in ((po.MODE_CANONICAL, "canonical"), (po.MODE_IGRAPH, "igraph")):
        t1 = time.perf_counter()
        olat, orel, ohops, ormin = og.routes(src[pick], hosts, mode, threads=threads)
        bad = ((bits(glat) != bits(olat)).any(axis=1) | (bits(grel) != bits(orel)).any(axis=1) |
               (ghops != ohops).any(axis=1) | (bits(grmin) != bits(ormin)))
        out[name] = {"rows_differing": int(bad.sum()), "oracle_s": round(time.perf_counter() - t1, 1),
                     "threads": threads}
        print(json.dumps(out), flush=True)
    ok = out["canonical"]["rows_differing"] == 0 and out["igraph"]["rows_differing"] == 0
    print(f"PARITY {'OK' if ok else 'MISMATCH'} ({label})", flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
