"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
checker / CPU baseline. The product (shadow_amd/) never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "liboracle.so")
_lib = None

P = C.POINTER
i32, i64, f64 = C.c_int32, C.c_int64, C.c_double


def build() -> None:
    subprocess.check_call(["make", "-s", "-C", _HERE])


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    lib = C.CDLL(LIB)
    lib.orc_graph_new.restype = C.c_void_p
    lib.orc_graph_new.argtypes = [i32, i64, C.c_int, P(i32), P(i32), P(f64), P(f64), P(f64)]
    lib.orc_graph_free.argtypes = [C.c_void_p]
    lib.orc_is_complete.argtypes = [C.c_void_p]
    lib.orc_get_eid.restype = i64
    lib.orc_get_eid.argtypes = [C.c_void_p, i32, i32]
    lib.orc_lookup_path.argtypes = [C.c_void_p, i32, i32, P(f64), P(f64)]
    lib.orc_epilogue.argtypes = [C.c_void_p, i32, P(i32), i32, P(f64), P(f64)]
    lib.orc_dijkstra.argtypes = [C.c_void_p, i32, P(i32), i32, P(f64), P(i64)]
    lib.orc_dijkstra_all.argtypes = [C.c_void_p, i32, P(f64), P(i64)]
    lib.orc_canonical_pred.argtypes = [C.c_void_p, P(f64), i32, P(i32), P(i32)]
    lib.orc_routes.argtypes = [C.c_void_p, P(i32), i32, P(i32), i32, C.c_int, P(f64), P(f64), P(i32), P(f64),
                               C.c_int]
    lib.orc_window_ns.restype = C.c_uint64
    lib.orc_window_ns.argtypes = [f64, C.c_uint64]
    lib.orc_delay_ns.restype = C.c_uint64
    lib.orc_delay_ns.argtypes = [f64]
    _lib = lib
    return lib


def _p(a, t):
    return a.ctypes.data_as(P(t))


MODE_IGRAPH = 0  # shortest-path branch, igraph-like heap parents
MODE_CANONICAL = 1  # shortest-path branch, tight predecessor with min (dist[u], index): igraph's rule + index on ties
MODE_COMPLETE = 2  # complete-graph branch (direct edge)


class OracleGraph:
    def __init__(self, V, efrom, eto, lat, loss, vloss, directed=False):
        self.lib = load()
        self.V = int(V)
        self._keep = [np.ascontiguousarray(efrom, np.int32), np.ascontiguousarray(eto, np.int32),
                      np.ascontiguousarray(lat, np.float64), np.ascontiguousarray(loss, np.float64),
                      np.ascontiguousarray(vloss, np.float64)]
        ef, et, la, lo, vl = self._keep
        self.E = len(ef)
        self.h = self.lib.orc_graph_new(self.V, self.E, int(directed), _p(ef, i32), _p(et, i32), _p(la, f64),
                                        _p(lo, f64), _p(vl, f64))
        if not self.h:
            raise ValueError("orc_graph_new failed")

    @classmethod
    def from_graph(cls, g):
        """From a shadow_amd.routes.Graph (its exported arrays)."""
        ef, et, lat, lo, vl = g.export()
        return cls(g.V, ef, et, lat, lo, vl, g.directed)

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.orc_graph_free(self.h)
            self.h = None

    def is_complete(self) -> bool:
        return bool(self.lib.orc_is_complete(self.h))

    def get_eid(self, u, v) -> int:
        return int(self.lib.orc_get_eid(self.h, int(u), int(v)))

    def lookup_path(self, s, t):
        lat, rel = C.c_double(), C.c_double()
        rc = self.lib.orc_lookup_path(self.h, int(s), int(t), C.byref(lat), C.byref(rel))
        return (lat.value, rel.value) if rc == 0 else None

    def epilogue(self, s, path):
        p = np.ascontiguousarray(path, np.int32)
        lat, rel = C.c_double(), C.c_double()
        rc = self.lib.orc_epilogue(self.h, int(s), _p(p, i32), len(p), C.byref(lat), C.byref(rel))
        return (lat.value, rel.value) if rc == 0 else None

    def dijkstra(self, s, targets=None):
        d = np.empty(self.V, np.float64)
        pe = np.empty(self.V, np.int64)
        if targets is None:
            self.lib.orc_dijkstra_all(self.h, int(s), _p(d, f64), _p(pe, i64))
        else:
            t = np.ascontiguousarray(targets, np.int32)
            self.lib.orc_dijkstra(self.h, int(s), _p(t, i32), len(t), _p(d, f64), _p(pe, i64))
        return d, pe

    def canonical_pred(self, s, dist):
        pred = np.empty(self.V, np.int32)
        nt = np.empty(self.V, np.int32)
        d = np.ascontiguousarray(dist, np.float64)
        self.lib.orc_canonical_pred(self.h, _p(d, f64), int(s), _p(pred, i32), _p(nt, i32))
        return pred, nt

    def routes(self, src, dst, mode, threads=1):
        s = np.ascontiguousarray(src, np.int32)
        t = np.ascontiguousarray(dst, np.int32)
        S, T = len(s), len(t)
        lat = np.empty((S, T), np.float64)
        rel = np.empty((S, T), np.float64)
        hops = np.empty((S, T), np.int32)
        rmin = np.empty(S, np.float64)
        self.lib.orc_routes(self.h, _p(s, i32), S, _p(t, i32), T, int(mode), _p(lat, f64), _p(rel, f64),
                            _p(hops, i32), _p(rmin, f64), int(threads))
        return lat, rel, hops, rmin


def window_ns(min_latency_ms: float, runahead_ns: int = 0) -> int:
    return int(load().orc_window_ns(float(min_latency_ms), int(runahead_ns)))


def delay_ns(latency_ms: float) -> int:
    return int(load().orc_delay_ns(float(latency_ms)))


def unique_mask(pred: np.ndarray, ntight: np.ndarray, dist: np.ndarray, s: int) -> np.ndarray:
    """uniq[v]: every vertex on v's canonical chain has exactly one tight predecessor."""
    V = len(pred)
    order = np.argsort(np.where(dist < 0, np.inf, dist), kind="stable")
    uniq = np.zeros(V, bool)
    uniq[s] = True
    for v in order:
        if v == s or dist[v] < 0:
            continue
        p = pred[v]
        uniq[v] = p >= 0 and ntight[v] == 1 and uniq[p]
    return uniq
