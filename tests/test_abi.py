"""C-ABI checks that need no GPU: the library loads, exports every symbol that
include/*.h declares, and fails loudly (no CPU fallback) without a device."""
import ctypes as C
import os
import re
import subprocess

import pytest

from shadow_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions(path):
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    txt = re.sub(r"//[^\n]*", "", txt)
    pat = r"\b((?:shdr|topology|address|random|worker|shdtop)_\w+)\s*\("
    return set(re.findall(pat, txt))


@pytest.mark.parametrize("header", ["shdr.h", "shd_topology.h"])
def test_every_declared_symbol_is_exported(header):
    names = header_functions(os.path.join(ROOT, "include", header))
    assert len(names) > 5
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH]).decode()
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    missing = sorted(n for n in names if n not in exported)
    assert not missing, missing
    # and the ctypes prototypes cover them
    assert not sorted(n for n in names if n not in _lib.PROTOTYPES)


def test_dropin_signatures_match_reference_header():
    """Same seven functions as /root/reference/src/main/routing/shd-topology.h:14-22."""
    names = header_functions(os.path.join(ROOT, "include", "shd_topology.h"))
    for fn in ("topology_new", "topology_free", "topology_attach", "topology_detach", "topology_isRoutable",
               "topology_getLatency", "topology_getReliability"):
        assert fn in names


def test_shadow_imports_are_weak():
    """address_*/random_nextDouble/worker_updateMinTimeJump must be overridable by Shadow."""
    out = subprocess.check_output(["nm", "-D", _lib.LIB_PATH]).decode()
    kinds = {ln.split()[-1]: ln.split()[-2] for ln in out.splitlines() if len(ln.split()) >= 2}
    for fn in ("address_toNetworkIP", "address_toHostIPString", "address_toString", "address_stringToIP",
               "random_nextDouble", "worker_updateMinTimeJump"):
        assert kinds.get(fn) in ("W", "V"), (fn, kinds.get(fn))


def test_no_gpu_fails_loudly():
    from shadow_amd.routes import Engine, Graph, ShdrError, device_count
    if device_count() > 0:
        pytest.skip("a GPU is visible")
    g = Graph.generate("ba", 500, 2, 1)
    with pytest.raises(ShdrError, match="no HIP device"):
        Engine(g)


def test_version_and_error_buffer():
    lib = _lib.load()
    assert b"gfx950" in lib.shdr_version()
    lib.shdr_graph_load_graphml(b"/nonexistent/file.graphml")
    assert "nonexistent" in _lib.last_error()


def test_oracle_is_not_linked_by_product():
    out = subprocess.check_output(["ldd", _lib.LIB_PATH]).decode()
    assert "oracle" not in out
    out = subprocess.check_output(["nm", "-D", _lib.LIB_PATH]).decode()
    assert "orc_" not in out
