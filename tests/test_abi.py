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


def header_prototypes(path):
    """{name: (return type, [parameter types])} of every function prototype in a C
    header, types normalised: comments, parameter names and whitespace dropped,
    pointer stars kept ("const gchar*", "guint64*")."""
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    txt = re.sub(r"//[^\n]*", "", txt)
    txt = re.sub(r"^\s*#.*$", "", txt, flags=re.M)
    out = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(\w+)\s*\(([^()]*)\)\s*;", txt):
        ret, name, params = m.group(1), m.group(2), m.group(3)
        if ret.strip().startswith(("typedef", "return")):
            continue

        def norm(t):
            t = re.sub(r"\s*\*\s*", "* ", t).strip()
            return re.sub(r"\s+", " ", t).replace("* ", "*").replace(" *", "*")

        types = []
        for p in params.split(","):
            tok = re.findall(r"\w+|\*", p)
            if not tok or tok == ["void"]:
                continue
            if len(tok) >= 2 and re.match(r"[A-Za-z_]", tok[-1]) and tok[-1] not in ("int", "char", "long", "double",
                                                                                  "float", "short", "const"):
                tok = tok[:-1]  # the parameter name
            types.append(norm(" ".join(tok)))
        out[name] = (norm(ret), types)
    return out


# shd-topology.h:14-22 of the reference, transcribed (the reference header is read
# directly as well when /root/reference is present).
REFERENCE_API = {
    "topology_new": ("Topology*", ["const gchar*"]),
    "topology_free": ("void", ["Topology*"]),
    "topology_attach": ("void", ["Topology*", "Address*", "Random*", "gchar*", "gchar*", "gchar*", "guint64*",
                                 "guint64*"]),
    "topology_detach": ("void", ["Topology*", "Address*"]),
    "topology_isRoutable": ("gboolean", ["Topology*", "Address*", "Address*"]),
    "topology_getLatency": ("gdouble", ["Topology*", "Address*", "Address*"]),
    "topology_getReliability": ("gdouble", ["Topology*", "Address*", "Address*"]),
}
REFERENCE_HEADER = "/root/reference/src/main/routing/shd-topology.h"


def test_header_parser_sees_types():
    protos = header_prototypes(os.path.join(ROOT, "include", "shd_topology.h"))
    assert protos["topology_attach"][1][3] == "gchar*"
    assert protos["shdtop_min_time_jump_history"] == ("uint64_t", ["gdouble*", "uint64_t"])


def test_dropin_signatures_match_reference_header():
    """The seven functions of shd-topology.h:14-22 with identical return and
    parameter types, arity and order (a type or arity drift fails here)."""
    mine = header_prototypes(os.path.join(ROOT, "include", "shd_topology.h"))
    for fn, sig in REFERENCE_API.items():
        assert mine.get(fn) == sig, (fn, mine.get(fn), sig)
    if os.path.exists(REFERENCE_HEADER):
        ref = header_prototypes(REFERENCE_HEADER)
        assert set(ref) == set(REFERENCE_API)
        for fn, sig in ref.items():
            assert mine.get(fn) == sig, (fn, mine.get(fn), sig)


_CTYPE_OF = {"void": None, "int": C.c_int, "gboolean": C.c_int, "int32_t": C.c_int32, "int64_t": C.c_int64,
             "uint32_t": C.c_uint32, "uint64_t": C.c_uint64, "guint64": C.c_uint64, "double": C.c_double,
             "gdouble": C.c_double, "float": C.c_float, "size_t": C.c_size_t, "unsigned int": C.c_uint}


def _ctype_ok(ctype, ctyp):
    """Does a ctypes argtype/restype faithfully represent C type `ctyp`?"""
    if ctyp.endswith("*"):
        base = ctyp.rstrip("*").replace("const ", "").strip()
        if base in ("char", "gchar") and ctyp.count("*") == 1:
            return ctype in (C.c_char_p, C.c_void_p)
        if ctype is C.c_void_p:
            return True  # opaque handles / buffers passed as addresses
        want = _CTYPE_OF.get(base)
        if want is not None:
            return getattr(ctype, "_type_", None) is want
        return hasattr(ctype, "_type_")  # pointer to a struct (shdr_graph_info) or char* array
    return ctype is _CTYPE_OF.get(ctyp.replace("const ", ""))


@pytest.mark.parametrize("header", ["shdr.h", "shd_topology.h"])
def test_ctypes_prototypes_match_header_types(header):
    """Every ctypes prototype the bindings use has the header's arity and types."""
    protos = header_prototypes(os.path.join(ROOT, "include", header))
    assert len(protos) > 5
    for name, (ret, params) in protos.items():
        res, args = _lib.PROTOTYPES[name]
        assert len(args) == len(params), (name, params, args)
        assert _ctype_ok(res, ret) if ret != "void" else res is None, (name, ret, res)
        for k, (a, p) in enumerate(zip(args, params)):
            assert _ctype_ok(a, p), (name, k, p, a)


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
