"""Host -> vertex attachment, restated from the reference — TEST INFRASTRUCTURE ONLY.

Used by tests/test_attach.py as the checker of the drop-in's topology_attach
(shadow_amd/csrc/topology.cpp). Pure Python over the GraphML vertex attributes;
the random source is libc rand_r exactly as Random uses it.

Follows /root/reference/src/main/routing/shd-topology.c:
  attach_hook      _topology_findAttachmentVertexHelperHook   :1071-1145
  longest_prefix   _topology_getLongestPrefixMatch            :1147-1172
  find_vertex      _topology_findAttachmentVertex             :1174-1258
and /root/reference/src/main/utility/shd-random.c:30-41 (random_nextDouble)
and shd-address.c:137-144 (address_stringToIP: inet_pton, else INADDR_NONE).
"""
from __future__ import annotations

import ctypes
import math
import socket
import struct

INADDR_NONE = 0xFFFFFFFF
INADDR_ANY = 0
_libc = ctypes.CDLL(None)
_libc.rand_r.argtypes = [ctypes.POINTER(ctypes.c_uint)]
_libc.rand_r.restype = ctypes.c_int
RAND_MAX = 2147483647  # glibc


class Random:
    """shd-random.c: a rand_r() seed state."""

    def __init__(self, seed: int):
        self.state = ctypes.c_uint(seed)

    def next_double(self) -> float:
        return float(_libc.rand_r(ctypes.byref(self.state))) / float(RAND_MAX)


def string_to_ip(s: str | None) -> int:
    """in_addr_t as stored in memory (network byte order read as a native u32)."""
    if s is None:
        return INADDR_NONE
    try:
        return struct.unpack("=I", socket.inet_pton(socket.AF_INET, s))[0]
    except OSError:
        return INADDR_NONE


def find_vertex(vertices, rnd: Random, ip_hint=None, geocode_hint=None, type_hint=None) -> int:
    """vertices: list of dicts with 'id', 'ip', 'geocode', 'type' in vertex-index order."""
    requested = string_to_ip(ip_hint) if ip_hint else INADDR_NONE
    q_all, q_type, q_code, q_tc = [], [], [], []
    n_all = n_type = n_code = n_tc = 0
    exact = False
    for v, a in enumerate(vertices):
        if "poi" not in a.get("id", ""):
            continue
        vip = string_to_ip(a.get("ip", ""))
        usable = vip not in (INADDR_NONE, INADDR_ANY)
        if ip_hint and requested not in (INADDR_NONE, INADDR_ANY) and vip == requested:
            if not exact:
                q_all, q_type, q_code, q_tc = [], [], [], []
            exact = True
            q_all.append(v)
            n_all += usable
        if exact:
            continue
        tm = type_hint is not None and a.get("type", "").lower() == type_hint.lower()
        cm = geocode_hint is not None and a.get("geocode", "").lower() == geocode_hint.lower()
        q_all.append(v)
        n_all += usable
        if tm:
            q_type.append(v)
            n_type += usable
        if cm:
            q_code.append(v)
            n_code += usable
        if tm and cm:
            q_tc.append(v)
            n_tc += usable
    if q_tc:
        cands, lpm = q_tc, bool(ip_hint) and n_tc > 0
    elif q_type:
        cands, lpm = q_type, bool(ip_hint) and n_type > 0
    elif q_code:
        cands, lpm = q_code, bool(ip_hint) and n_code > 0
    else:
        cands, lpm = q_all, bool(ip_hint) and n_all > 0
    if not cands:
        return -1
    if lpm and not exact:
        best, best_v = 0, -1
        for v in cands:
            m = string_to_ip(vertices[v].get("ip", "")) & requested
            if m > best:
                best, best_v = m, v
        return best_v
    x = float(len(cands) - 1) * rnd.next_double()
    chosen = math.floor(x)
    if x - chosen >= 0.5:  # C round(): halves away from zero (x >= 0 here)
        chosen += 1
    return cands[int(chosen)]
