"""ctypes binding of libshdtopology.so (include/shdr.h, include/shd_topology.h).

The library is built in-tree by ``make -C shadow_amd`` (``__graft_entry__.build``).
There is no Python or CPU fallback for route computation: if the shared object
is missing, importing this module raises, and on a host without a gfx950 GPU
``shdr_engine_create`` fails with SHDR_ENODEV.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# SHDR_LIB_VARIANT=diag selects the diagnostic build (make -C shadow_amd diag)
_FLAVOR = os.environ.get("SHDR_LIB_VARIANT", "")  # experiment builds: make -C shadow_amd flavor NAME=...
LIB_PATH = os.path.join(_HERE, f"libshdtopology_{_FLAVOR}.so" if _FLAVOR else "libshdtopology.so")

i32, i64, u32, u64, f64 = C.c_int32, C.c_int64, C.c_uint32, C.c_uint64, C.c_double
vp, cp = C.c_void_p, C.c_char_p
P = C.POINTER

SHDR_OK = 0
SHDR_OUT_DEVICE = 0x1
SHDR_FORCE_SSSP = 0x2
SHDR_TIMING = 0x4
SHDR_KEEP_TREES = 0x8
SHDR_PATH_JITTER = 0x10


class GraphInfo(C.Structure):
    _fields_ = [
        ("vertex_count", i32),
        ("edge_count", i64),
        ("is_directed", i32),
        ("is_connected", i32),
        ("cluster_count", i32),
        ("is_complete", i32),
        ("self_loops", i64),
        ("bad_latency_edges", i64),
    ]


# name -> (restype, argtypes); every symbol declared in include/*.h
PROTOTYPES = {
    # shdr.h
    "shdr_graph_load_graphml": (vp, [cp]),
    "shdr_graph_parse_graphml": (vp, [cp, C.c_size_t]),
    "shdr_graph_from_edges": (vp, [i32, i64, i32, P(i32), P(i32), P(f64), P(f64), P(f64)]),
    "shdr_graph_generate": (vp, [i32, i32, i32, u64]),
    "shdr_graph_save_binary": (C.c_int, [vp, cp]),
    "shdr_graph_load_binary": (vp, [cp]),
    "shdr_graph_save_graphml": (C.c_int, [vp, cp]),
    "shdr_graph_free": (None, [vp]),
    "shdr_graph_check": (C.c_int, [vp, P(GraphInfo)]),
    "shdr_graph_vertex_count": (i32, [vp]),
    "shdr_graph_edge_count": (i64, [vp]),
    "shdr_graph_is_directed": (i32, [vp]),
    "shdr_graph_vertex_num": (f64, [vp, cp, i32]),
    "shdr_graph_vertex_str": (cp, [vp, cp, i32]),
    "shdr_graph_edge_num": (f64, [vp, cp, i64]),
    "shdr_graph_edge_ends": (C.c_int, [vp, i64, P(i32), P(i32)]),
    "shdr_graph_export_edges": (C.c_int, [vp, P(i32), P(i32), P(f64), P(f64), P(f64)]),
    "shdr_graph_get_eid": (i64, [vp, i32, i32]),
    "shdr_engine_create": (vp, [vp, i32]),
    "shdr_engine_free": (None, [vp]),
    "shdr_routes_compute": (C.c_int, [vp, vp, i32, vp, i32, vp, vp, vp, vp, u32, vp]),
    "shdr_engine_pred_tree": (C.c_int, [vp, i32, P(i32), P(f64)]),
    "shdr_engine_partition": (C.c_int, [vp, P(i32), i32, i32, P(i32)]),
    "shdr_engine_timing": (C.c_int, [vp, P(i32), P(cp), P(C.c_float), i32]),
    "shdr_engine_last_layout": (C.c_int, [vp, P(i32), i32]),
    "shdr_engine_row_order": (i32, [vp, P(i32), i32]),
    "shdr_engine_set_delta": (C.c_int, [vp, f64]),
    "shdr_engine_set_variant": (C.c_int, [vp, i32]),
    "shdr_write_complete_graphml": (C.c_int, [vp, P(i32), i32, P(f64), P(f64), cp]),
    "shdr_device_count": (i32, []),
    "shdr_last_error": (C.c_int, [cp, C.c_size_t]),
    "shdr_version": (cp, []),
    # shd_topology.h (drop-in API + imported Shadow symbols + harness helpers)
    "topology_new": (vp, [cp]),
    "topology_free": (None, [vp]),
    "topology_attach": (None, [vp, vp, vp, cp, cp, cp, P(u64), P(u64)]),
    "topology_detach": (None, [vp, vp]),
    "topology_isRoutable": (C.c_int, [vp, vp, vp]),
    "topology_getLatency": (f64, [vp, vp, vp]),
    "topology_getReliability": (f64, [vp, vp, vp]),
    "address_toNetworkIP": (u32, [vp]),
    "address_toHostIPString": (cp, [vp]),
    "address_toString": (cp, [vp]),
    "address_stringToIP": (u32, [cp]),
    "random_nextDouble": (f64, [vp]),
    "worker_updateMinTimeJump": (None, [f64]),
    "shdtop_address_new": (vp, [u32, cp]),
    "shdtop_address_free": (None, [vp]),
    "shdtop_random_new": (vp, [C.c_uint]),
    "shdtop_random_free": (None, [vp]),
    "shdtop_last_min_time_jump": (f64, []),
    "shdtop_min_time_jump_calls": (u64, []),
    "shdtop_reset_min_time_jump": (None, []),
    "shdtop_min_time_jump_history": (u64, [P(f64), u64]),
    "topology_debug_isComplete": (C.c_int, [vp]),
    "topology_debug_isDirected": (C.c_int, [vp]),
    "topology_debug_minimumPathLatency": (f64, [vp]),
    "topology_debug_vertexOf": (i32, [vp, vp]),
    "topology_debug_lastComputeTimes": (C.c_int, [vp, P(f64), C.c_int]),
    "topology_debug_tableBlocks": (C.c_int, [vp, P(i32), P(i32)]),
}

_lib = None


def load() -> C.CDLL:
    """Load the in-tree library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: torch wheels bundle their own libamdhip64.so
    # (same SONAME as /opt/rocm's). Import torch first, when present, so that
    # this library binds to the runtime torch will use too.
    if os.environ.get("SHDR_NO_TORCH_PRELOAD") != "1":
        try:
            import torch  # noqa: F401
        except Exception:
            pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make -C {_HERE}` or __graft_entry__.build(); "
            "the routing engine has no fallback"
        )
    lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    for name, (res, args) in PROTOTYPES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if hasattr(lib, "shdr_diag_read"):
        lib.shdr_diag_read.restype = C.c_int
        lib.shdr_diag_read.argtypes = [P(C.c_ulonglong), C.c_int, C.c_int]
    _lib = lib
    return lib


def last_error() -> str:
    lib = load()
    buf = C.create_string_buffer(1024)
    lib.shdr_last_error(buf, len(buf))
    return buf.value.decode(errors="replace")


class ShdrError(RuntimeError):
    pass


def check(rc: int, what: str) -> None:
    if rc != SHDR_OK:
        raise ShdrError(f"{what} failed ({rc}): {last_error()}")
