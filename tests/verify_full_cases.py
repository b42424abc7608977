"""BASELINE-size relaxation postconditions through the verify flavour
(libshdtopology_verify.so, built with -DSHDR_VERIFY by `make -C shadow_amd flavor
NAME=verify DEFS=-DSHDR_VERIFY`; tests/conftest.py keeps it at the tree's sources).

Started by tests/test_gpu_verify.py in a fresh process with SHDR_LIB_VARIANT=verify
(one library per process). After every bucket's relaxation the flavour checks on the
device, for every lane of every vertex, that no pending word is left set (guard 128)
and that no arc improves its head (dist[h] <= fl(dist[v] + w) bitwise: guard 512), so
every distance of the WHOLE table is at the relaxation's fixed point — the tables
the suite samples row by row against the oracle, checked here in full. A tripped
guard makes shdr_routes_compute fail, which raises. Every slot runs buckets of both
row encodings (the no-fill parities) over the passes below.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import make_workload  # noqa: E402
from shadow_amd import _lib  # noqa: E402
from shadow_amd.routes import Engine, lib_kernel_sha, src_kernel_sha  # noqa: E402


def passes(eng, rows, hosts, n, label):
    dev = torch.device("cuda", 0)
    S, T = len(rows), len(hosts)
    lat = torch.empty((S, T), dtype=torch.float64, device=dev)
    rel = torch.empty((S, T), dtype=torch.float64, device=dev)
    rmin = torch.empty((S,), dtype=torch.float64, device=dev)
    for i in range(n):
        t0 = time.perf_counter()
        eng.compute_device(rows, hosts, lat.data_ptr(), rel.data_ptr(), rmin.data_ptr(), None)  # raises on a guard
        lay = eng.last_layout()
        assert lay["cluster_fallbacks_total"] == 0, lay
        print(f"verify ok: {label} pass {i} ({S} x {T}) {time.perf_counter() - t0:.1f} s layout {lay}", flush=True)
    del lat, rel, rmin
    torch.cuda.empty_cache()


def main() -> int:
    assert _lib.LIB_PATH.endswith("libshdtopology_verify.so"), _lib.LIB_PATH
    assert lib_kernel_sha() == src_kernel_sha(), (lib_kernel_sha(), src_kernel_sha())
    n = 0
    g, hosts, _, _ = make_workload("cfg4")
    eng = Engine(g)
    passes(eng, hosts, hosts, 2, "cfg4 full table")
    n += 1
    part = eng.partition(hosts, 8)
    for p in range(8):  # the 8-GPU shards: 3-wide PM 2 clusters on a 256-CU device
        passes(eng, hosts[part == p], hosts, 1, f"cfg4 shard {p} of 8")
        n += 1
    del eng
    g, hosts, _, _ = make_workload("cfg5")
    eng = Engine(g)
    passes(eng, hosts, hosts, 2, "cfg5 full table")
    n += 1
    print(f"verify full cases: {n} passed", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
