"""Host-side interface to the MI355X routing engine (the shdr_* C-ABI).

``Graph`` wraps a host topology (GraphML, plain edge arrays or a synthetic
generator); ``Engine`` uploads it to one GPU's HBM and computes route tables.
This module only marshals pointers: every byte of route arithmetic runs in the
HIP kernels of ``csrc/routes.hip``.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import (SHDR_FORCE_SSSP, SHDR_KEEP_TREES, SHDR_OUT_DEVICE, SHDR_TIMING, GraphInfo, ShdrError, check,
                   last_error)

__all__ = ["Graph", "Engine", "RouteTable", "device_count", "ShdrError", "SHDR_FORCE_SSSP", "SHDR_KEEP_TREES",
           "SHDR_TIMING", "SHDR_OUT_DEVICE"]


def _ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


def device_count() -> int:
    return int(_lib.load().shdr_device_count())


# the library's sources in the order shadow_amd/Makefile (LIB_SRCS) hashes them
LIB_SOURCES = ("csrc/routes.hip", "csrc/topology.cpp", "csrc/graph.cpp", "csrc/graph.hpp", "csrc/complete.cpp",
               "csrc/shim.c", "csrc/version.c", "../include/shdr.h", "../include/shd_topology.h")


def lib_kernel_sha(lib=None) -> str:
    """SHA-256 prefix (16 hex digits) of the sources the loaded library (or `lib`, a
    loaded flavour) was compiled from (shdr_version(), set by shadow_amd/Makefile):
    the kernel (routes.hip) and the host code around it (topology.cpp, graph.cpp, ...)."""
    v = (lib or _lib.load()).shdr_version().decode()
    return v.rsplit(" ", 1)[-1] if " kernel " in v else "unknown"


def src_kernel_sha() -> str:
    """The same prefix for the library sources as they are on disk now."""
    import hashlib
    import os
    d = os.path.dirname(os.path.abspath(__file__))
    h = hashlib.sha256()
    for f in LIB_SOURCES:
        h.update(open(os.path.join(d, f), "rb").read())
    return h.hexdigest()[:16]


class Graph:
    """Topology graph in host memory (igraph-equivalent indexing)."""

    def __init__(self, handle: int):
        if not handle:
            raise ShdrError(last_error())
        self._h = handle
        self._lib = _lib.load()

    # ---- constructors
    @classmethod
    def load_graphml(cls, path: str) -> "Graph":
        return cls(_lib.load().shdr_graph_load_graphml(str(path).encode()))

    @classmethod
    def load_binary(cls, path: str) -> "Graph":
        return cls(_lib.load().shdr_graph_load_binary(str(path).encode()))

    def save_binary(self, path: str) -> None:
        check(self._lib.shdr_graph_save_binary(self._h, str(path).encode()), "shdr_graph_save_binary")

    def save_graphml(self, path: str) -> None:
        """Lossless GraphML (load_graphml gives back the same graph)."""
        check(self._lib.shdr_graph_save_graphml(self._h, str(path).encode()), "shdr_graph_save_graphml")

    @classmethod
    def parse_graphml(cls, text: str | bytes) -> "Graph":
        b = text.encode() if isinstance(text, str) else text
        return cls(_lib.load().shdr_graph_parse_graphml(b, len(b)))

    @classmethod
    def from_edges(cls, V: int, efrom, eto, latency, loss=None, vloss=None, directed: bool = False) -> "Graph":
        efrom = np.ascontiguousarray(efrom, dtype=np.int32)
        eto = np.ascontiguousarray(eto, dtype=np.int32)
        lat = np.ascontiguousarray(latency, dtype=np.float64)
        E = len(efrom)
        lo = np.ascontiguousarray(loss if loss is not None else np.zeros(E), dtype=np.float64)
        vl = np.ascontiguousarray(vloss if vloss is not None else np.zeros(V), dtype=np.float64)
        h = _lib.load().shdr_graph_from_edges(int(V), int(E), int(bool(directed)), _ptr(efrom, C.c_int32),
                                              _ptr(eto, C.c_int32), _ptr(lat, C.c_double), _ptr(lo, C.c_double),
                                              _ptr(vl, C.c_double))
        return cls(h)

    @classmethod
    def generate(cls, kind: str, n: int, m: int = 3, seed: int = 1) -> "Graph":
        k = {"ba": 0, "chunglu": 1}[kind]
        return cls(_lib.load().shdr_graph_generate(k, int(n), int(m), int(seed)))

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._lib.shdr_graph_free(h)

    @property
    def handle(self) -> int:
        return self._h

    # ---- properties
    @property
    def V(self) -> int:
        return int(self._lib.shdr_graph_vertex_count(self._h))

    @property
    def E(self) -> int:
        return int(self._lib.shdr_graph_edge_count(self._h))

    @property
    def directed(self) -> bool:
        return bool(self._lib.shdr_graph_is_directed(self._h))

    def check(self) -> GraphInfo:
        info = GraphInfo()
        check(self._lib.shdr_graph_check(self._h, C.byref(info)), "shdr_graph_check")
        return info

    def vertex_num(self, attr: str, v: int) -> float:
        return float(self._lib.shdr_graph_vertex_num(self._h, attr.encode(), int(v)))

    def vertex_str(self, attr: str, v: int) -> str:
        return self._lib.shdr_graph_vertex_str(self._h, attr.encode(), int(v)).decode()

    def edge_num(self, attr: str, e: int) -> float:
        return float(self._lib.shdr_graph_edge_num(self._h, attr.encode(), int(e)))

    def get_eid(self, u: int, v: int) -> int:
        return int(self._lib.shdr_graph_get_eid(self._h, int(u), int(v)))

    def export(self):
        """(efrom, eto, latency, edge loss, vertex loss) as numpy arrays."""
        V, E = self.V, self.E
        ef = np.empty(E, np.int32)
        et = np.empty(E, np.int32)
        lat = np.empty(E, np.float64)
        lo = np.empty(E, np.float64)
        vl = np.empty(V, np.float64)
        check(self._lib.shdr_graph_export_edges(self._h, _ptr(ef, C.c_int32), _ptr(et, C.c_int32),
                                                 _ptr(lat, C.c_double), _ptr(lo, C.c_double), _ptr(vl, C.c_double)),
              "shdr_graph_export_edges")
        return ef, et, lat, lo, vl


@dataclass
class RouteTable:
    src: np.ndarray
    dst: np.ndarray
    lat: np.ndarray  # [S, T] ms
    rel: np.ndarray  # [S, T]
    hops: np.ndarray | None
    row_min: np.ndarray  # [S]


class Engine:
    """One GPU's copy of the graph plus the routing kernels."""

    def __init__(self, graph: Graph, device: int = 0):
        self._lib = _lib.load()
        self.graph = graph  # keep alive
        self.device = device
        self._h = self._lib.shdr_engine_create(graph.handle, int(device))
        if not self._h:
            raise ShdrError(last_error())

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._lib.shdr_engine_free(h)

    def set_delta(self, delta: float) -> None:
        check(self._lib.shdr_engine_set_delta(self._h, float(delta)), "shdr_engine_set_delta")

    def set_variant(self, variant: int) -> None:
        check(self._lib.shdr_engine_set_variant(self._h, int(variant)), "shdr_engine_set_variant")

    def compute(self, src, dst, *, hops: bool = False, flags: int = 0) -> RouteTable:
        """Route table into host numpy arrays."""
        src = np.ascontiguousarray(src, dtype=np.int32)
        dst = np.ascontiguousarray(dst, dtype=np.int32)
        S, T = len(src), len(dst)
        lat = np.empty((S, T), np.float64)
        rel = np.empty((S, T), np.float64)
        hp = np.empty((S, T), np.int32) if hops else None
        rmin = np.empty(S, np.float64)
        rc = self._lib.shdr_routes_compute(self._h, src.ctypes.data, S, dst.ctypes.data, T, lat.ctypes.data,
                                           rel.ctypes.data, hp.ctypes.data if hp is not None else None,
                                           rmin.ctypes.data, int(flags) & ~SHDR_OUT_DEVICE, None)
        check(rc, "shdr_routes_compute")
        return RouteTable(src, dst, lat, rel, hp, rmin)

    def compute_device(self, src, dst, lat_ptr: int, rel_ptr: int, row_min_ptr: int | None = None,
                       hops_ptr: int | None = None, *, flags: int = 0, stream: int | None = None) -> None:
        """Route table into caller-owned device buffers (e.g. torch tensors'
        data_ptr()) on this engine's GPU, launched on ``stream``."""
        src = np.ascontiguousarray(src, dtype=np.int32)
        dst = np.ascontiguousarray(dst, dtype=np.int32)
        rc = self._lib.shdr_routes_compute(self._h, src.ctypes.data, len(src), dst.ctypes.data, len(dst), lat_ptr,
                                           rel_ptr, hops_ptr, row_min_ptr, int(flags) | SHDR_OUT_DEVICE, stream)
        check(rc, "shdr_routes_compute")

    def pred_tree(self, i: int):
        """(pred_vertex[V], dist[V]) of source row i of the last compute made
        with SHDR_KEEP_TREES."""
        V = self.graph.V
        pred = np.empty(V, np.int32)
        dist = np.empty(V, np.float64)
        check(self._lib.shdr_engine_pred_tree(self._h, int(i), _ptr(pred, C.c_int32), _ptr(dist, C.c_double)),
              "shdr_engine_pred_tree")
        return pred, dist

    def partition(self, src, nparts: int) -> np.ndarray:
        """part[i] in [0, nparts): a balanced, spatially coherent split of the
        source list for strong scaling (identical on every engine of this graph)."""
        src = np.ascontiguousarray(src, dtype=np.int32)
        part = np.empty(len(src), np.int32)
        check(self._lib.shdr_engine_partition(self._h, _ptr(src, C.c_int32), len(src), int(nparts),
                                              _ptr(part, C.c_int32)), "shdr_engine_partition")
        return part

    def timing(self) -> dict[str, float]:
        n = C.c_int32(0)
        names = (C.c_char_p * 16)()
        ms = (C.c_float * 16)()
        check(self._lib.shdr_engine_timing(self._h, C.byref(n), names, ms, 16), "shdr_engine_timing")
        return {names[i].decode(): float(ms[i]) for i in range(min(n.value, 16))}

    def last_layout(self) -> dict[str, int]:
        """Bucket layout of the last shortest-path compute (shdr_engine_last_layout)."""
        out = (C.c_int32 * 10)()
        check(self._lib.shdr_engine_last_layout(self._h, out, 10), "shdr_engine_last_layout")
        return dict(zip(["variant", "cluster", "balanced", "rows_main", "tail_cluster", "partial_first",
                         "cluster_fallback", "cluster_fallbacks_total", "progressive", "tail_mode"], list(out)))

    def row_order(self) -> np.ndarray:
        """order[k] = caller row of the k-th source the last compute processed;
        order[:rows_main] ran in the main launch, the rest in the tail launch."""
        n = int(self._lib.shdr_engine_row_order(self._h, None, 0))
        if n < 0:
            raise ShdrError(last_error())
        out = np.empty(n, np.int32)
        if n:
            check(min(0, int(self._lib.shdr_engine_row_order(self._h, _ptr(out, C.c_int32), n))),
                  "shdr_engine_row_order")
        return out
