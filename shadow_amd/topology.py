"""Python mirror of Shadow's routing API over the drop-in C library.

Same names, argument meaning and error behaviour as
/root/reference/src/main/routing/shd-topology.h:14-22 (topology_new returns
None on failure; queries return -1.0 when a host is not attached or no path
exists). Addresses and Random objects are the standalone harness's
(shdtop_address_new / shdtop_random_new), keyed by IPv4 string as Shadow's
DNS assigns them (11.0.0.0 and up, shd-dns.c:94-104).
"""
from __future__ import annotations

import ctypes as C
import socket
import struct

from . import _lib


def ip_to_network(ip: str) -> int:
    """dotted quad -> in_addr_t (network byte order), as inet_pton."""
    return struct.unpack("=I", socket.inet_aton(ip))[0]


class Address:
    def __init__(self, ip: str, name: str = "host"):
        self._lib = _lib.load()
        self.ip = ip
        self._h = self._lib.shdtop_address_new(ip_to_network(ip), name.encode())

    @property
    def handle(self):
        return self._h

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._lib.shdtop_address_free(h)


class Random:
    """shd-random.c: rand_r() over a seed state."""

    def __init__(self, seed: int):
        self._lib = _lib.load()
        self._h = self._lib.shdtop_random_new(int(seed))

    @property
    def handle(self):
        return self._h

    def next_double(self) -> float:
        return float(self._lib.random_nextDouble(self._h))

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._lib.shdtop_random_free(h)


class Topology:
    """topology_new / attach / detach / getLatency / getReliability / isRoutable."""

    def __init__(self, handle):
        self._lib = _lib.load()
        self._h = handle

    @classmethod
    def new(cls, graph_path: str) -> "Topology | None":
        h = _lib.load().topology_new(str(graph_path).encode())
        return cls(h) if h else None

    def free(self) -> None:
        h, self._h = self._h, None
        if h:
            self._lib.topology_free(h)

    def __del__(self):
        if getattr(self, "_h", None):
            self.free()

    def attach(self, address: Address, rnd: Random, ip_hint: str | None = None, geocode_hint: str | None = None,
               type_hint: str | None = None) -> tuple[int, int]:
        bw_down = C.c_uint64(0)
        bw_up = C.c_uint64(0)
        enc = lambda s: s.encode() if s is not None else None  # noqa: E731
        self._lib.topology_attach(self._h, address.handle, rnd.handle, enc(ip_hint), enc(geocode_hint),
                                  enc(type_hint), C.byref(bw_down), C.byref(bw_up))
        return bw_down.value, bw_up.value

    def detach(self, address: Address) -> None:
        self._lib.topology_detach(self._h, address.handle)

    def get_latency(self, src: Address, dst: Address) -> float:
        return float(self._lib.topology_getLatency(self._h, src.handle, dst.handle))

    def get_reliability(self, src: Address, dst: Address) -> float:
        return float(self._lib.topology_getReliability(self._h, src.handle, dst.handle))

    def is_routable(self, src: Address, dst: Address) -> bool:
        return bool(self._lib.topology_isRoutable(self._h, src.handle, dst.handle))

    # introspection
    @property
    def is_complete(self) -> bool:
        return bool(self._lib.topology_debug_isComplete(self._h))

    @property
    def is_directed(self) -> bool:
        return bool(self._lib.topology_debug_isDirected(self._h))

    @property
    def minimum_path_latency(self) -> float:
        return float(self._lib.topology_debug_minimumPathLatency(self._h))

    def vertex_of(self, address: Address) -> int:
        return int(self._lib.topology_debug_vertexOf(self._h, address.handle))

    def last_compute_times(self) -> dict:
        """Phases of the last table computation (topology_debug_lastComputeTimes)."""
        out = (C.c_double * 9)()
        self._lib.topology_debug_lastComputeTimes(self._h, out, 9)
        keys = ["engine_create_ms", "block_ms", "block_rows", "landmarks_ms", "grouping_ms", "launch_ms", "pass_ms",
                "d2h_ms", "engine_total_ms"]
        return dict(zip(keys, list(out)))

    def table_blocks(self) -> tuple[int, int, int]:
        """(blocks, rows per block, computed blocks) of the current table."""
        rows, done = C.c_int32(0), C.c_int32(0)
        n = self._lib.topology_debug_tableBlocks(self._h, C.byref(rows), C.byref(done))
        return int(n), int(rows.value), int(done.value)


def last_min_time_jump() -> float:
    """Last value the (standalone shim) worker_updateMinTimeJump upcall received."""
    return float(_lib.load().shdtop_last_min_time_jump())


def min_time_jump_calls() -> int:
    return int(_lib.load().shdtop_min_time_jump_calls())


def reset_min_time_jump() -> None:
    _lib.load().shdtop_reset_min_time_jump()


def min_time_jump_history(cap: int = 4096) -> list[float]:
    """Upcall values in call order (the shim records the first 4096)."""
    buf = (C.c_double * cap)()
    n = int(_lib.load().shdtop_min_time_jump_history(buf, cap))
    return [float(buf[i]) for i in range(min(n, cap))]
