"""Offline all-sources precompute on MI355X: sparse topology -> complete topology.

SURVEY §8(f) row 3. Replaces /root/reference/src/tools/topology/compute-topology-paths.py
(step 3 of the map pipeline in src/tools/topology/readme:1-4): for every pair of
points of interest, the shortest-path latency and the mean per-hop jitter, written
as a complete undirected GraphML that the simulator then serves through its
isComplete branch (direct edge, no shortest paths at run time).

The reference runs one networkx Dijkstra per source in a process pool
(:46-84) and builds the output graph in Python. Here:
  * the P x P metrics are ONE engine call per GPU on the route-table kernel with
    SHDR_PATH_JITTER (the pred entries carry per-arc jitter, folded by sum in
    path order, include/shdr.h); rows are split over GPUs, one engine each;
  * the GraphML is formatted natively (shdr_write_complete_graphml), row-parallel.

Differences, by design:
  * point-of-interest selection (:133-155) is seeded and ordered by vertex index
    (the tool samples a Python set, so its order and sample vary run to run);
    a sample larger than the client count takes every client (the tool raises);
  * ties between equal-latency paths follow the engine's canonical rule
    (minimum-index tight in-arc) rather than networkx's heap order.

CLI:  python -m shadow_amd.complete_topology IN.graphml[.xz] OUT.graphml
          [--sample 10000] [--seed 1] [--all] [--gpus N]
"""
from __future__ import annotations

import argparse
import ctypes as C
import lzma
import os
import sys
import tempfile
import threading
import time

import numpy as np

from . import _lib
from ._lib import SHDR_PATH_JITTER, check
from .routes import Engine, Graph

CLIENT_SAMPLE_SIZE = 10000  # compute-topology-paths.py:11


def select_pois(g: Graph, sample: int = CLIENT_SAMPLE_SIZE, seed: int = 1) -> np.ndarray:
    """compute-topology-paths.py:133-155: relays, servers, a sample of clients and
    one client for every geocode the sample misses. -> sorted vertex indices."""
    relays, servers, clients = [], [], []
    for v in range(g.V):
        t = g.vertex_str("type", v)
        if t == "relay":
            relays.append(v)
        elif t == "server":
            servers.append(v)
        elif t == "client":
            clients.append(v)
    codes = {}
    for v in clients:  # the last client seen represents its geocode
        codes[g.vertex_str("geocode", v)] = v
    rng = np.random.default_rng(seed)
    n = min(sample, len(clients))
    chosen = set(int(x) for x in rng.choice(np.asarray(clients, dtype=np.int64), size=n, replace=False)) if n else set()
    for v in chosen:
        codes.pop(g.vertex_str("geocode", v), None)
    chosen.update(codes.values())
    return np.array(sorted(chosen.union(servers, relays)), dtype=np.int32)


def path_tables(g: Graph, pois: np.ndarray, devices=(0,)) -> tuple[np.ndarray, np.ndarray]:
    """-> (lat[P,P], jit[P,P]) f64: row i = paths from pois[i]; rows split over `devices`."""
    pois = np.ascontiguousarray(pois, dtype=np.int32)
    P = len(pois)
    lat = np.empty((P, P), np.float64)
    jit = np.empty((P, P), np.float64)
    devices = list(devices)[:max(1, P)]
    bounds = np.linspace(0, P, len(devices) + 1).astype(int)
    errors = []

    def run(k, dev):
        lo, hi = bounds[k], bounds[k + 1]
        if hi <= lo:
            return
        try:
            t = Engine(g, device=dev).compute(pois[lo:hi], pois, flags=SHDR_PATH_JITTER)
            lat[lo:hi] = t.lat
            jit[lo:hi] = t.rel
        except Exception as e:  # re-raised in the caller's thread
            errors.append(e)

    threads = [threading.Thread(target=run, args=(k, d)) for k, d in enumerate(devices)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        raise errors[0]
    return lat, jit


def write_complete(g: Graph, pois: np.ndarray, lat: np.ndarray, jit: np.ndarray, path: str) -> None:
    pois = np.ascontiguousarray(pois, dtype=np.int32)
    lat = np.ascontiguousarray(lat, dtype=np.float64)
    jit = np.ascontiguousarray(jit, dtype=np.float64)
    P = len(pois)
    if lat.shape != (P, P) or jit.shape != (P, P):
        raise ValueError("lat/jit must be P x P")
    f64p = C.POINTER(C.c_double)
    rc = _lib.load().shdr_write_complete_graphml(g.handle, pois.ctypes.data_as(C.POINTER(C.c_int32)), P,
                                                 lat.ctypes.data_as(f64p), jit.ctypes.data_as(f64p),
                                                 str(path).encode())
    check(rc, "shdr_write_complete_graphml")


def load_any(path: str) -> Graph:
    if not path.endswith(".xz"):
        return Graph.load_graphml(path)
    with tempfile.NamedTemporaryFile(suffix=".graphml.xml") as f:
        f.write(lzma.open(path).read())
        f.flush()
        return Graph.load_graphml(f.name)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("input")
    ap.add_argument("output")
    ap.add_argument("--sample", type=int, default=CLIENT_SAMPLE_SIZE, help="clients sampled (tool default 10000)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--all", action="store_true", help="every vertex is a point of interest")
    ap.add_argument("--gpus", type=int, default=1)
    a = ap.parse_args(argv)
    t0 = time.perf_counter()
    g = load_any(a.input)
    pois = np.arange(g.V, dtype=np.int32) if a.all else select_pois(g, a.sample, a.seed)
    t1 = time.perf_counter()
    lat, jit = path_tables(g, pois, range(a.gpus))
    t2 = time.perf_counter()
    write_complete(g, pois, lat, jit, a.output)
    t3 = time.perf_counter()
    print(f"{len(pois)} points of interest: load {t1 - t0:.2f} s, paths {t2 - t1:.2f} s on {a.gpus} GPU(s), "
          f"write {t3 - t2:.2f} s ({os.path.getsize(a.output) / 1e6:.1f} MB)", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
