"""shadow_amd — MI355X-native topology routing for the Shadow simulator.

Drop-in for Shadow's routing hot path (src/main/routing/shd-topology.c):
``libshdtopology.so`` exports the reference's C API (include/shd_topology.h)
and the device C-ABI (include/shdr.h); the HIP kernels live in
``csrc/routes.hip``. Python modules here are thin ctypes wrappers used by
tests and bench.py.
"""
from ._lib import LIB_PATH, ShdrError, load  # noqa: F401

__version__ = "0.1.0"
