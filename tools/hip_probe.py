#!/usr/bin/env python3
"""Bare HIP runtime probe (no repository library loaded): hipGetDeviceCount and a
1-byte device allocation. Run first in a GPU session so that a card handed over in
a faulted state is told apart from a fault of this repository's kernels."""
import ctypes
import sys

hip = ctypes.CDLL("libamdhip64.so")
hip.hipGetErrorString.restype = ctypes.c_char_p
n = ctypes.c_int(-1)
rc = hip.hipGetDeviceCount(ctypes.byref(n))
print(f"hipGetDeviceCount rc={rc} ({hip.hipGetErrorString(rc).decode()}) n={n.value}", flush=True)
if rc != 0:
    sys.exit(3)
p = ctypes.c_void_p()
rc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1))
print(f"hipMalloc rc={rc} ({hip.hipGetErrorString(rc).decode()})", flush=True)
if rc == 0:
    hip.hipFree(p)
sys.exit(0 if rc == 0 else 3)
