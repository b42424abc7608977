import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


# the in-tree library flavours: file -> make arguments (shadow_amd/Makefile)
FLAVOURS = {
    "libshdtopology.so": ["all"],
    "libshdtopology_bchk.so": ["bchk"],  # bounds-checked (tests/test_gpu_bchk.py)
    "libshdtopology_exp.so": ["flavor", "NAME=exp", "DEFS=-DSHDR_EXPERIMENTS"],  # schedule knobs
    "libshdtopology_verify.so": ["flavor", "NAME=verify", "DEFS=-DSHDR_VERIFY"],  # fixed-point checks
}
_VERSION_TAG = b"(gfx950) kernel "


def built_sha(path: str) -> str | None:
    """The source sha compiled into a library file (shdr_version's string in its
    read-only data; no load, no GPU), or None if the file is missing."""
    if not os.path.exists(path):
        return None
    data = open(path, "rb").read()
    i = data.find(_VERSION_TAG)
    return data[i + len(_VERSION_TAG):i + len(_VERSION_TAG) + 16].decode(errors="replace") if i >= 0 else "unknown"


def tree_sha() -> str:
    from shadow_amd.routes import src_kernel_sha
    return src_kernel_sha()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    # build every in-tree library flavour that a fresh checkout lacks or that was
    # compiled from other sources than the tree's (CPU-only step), so no test can run
    # a kernel older than the tree (the flavour tests assert the sha again)
    want = tree_sha()
    d = os.path.join(ROOT, "shadow_amd")
    for so, args in FLAVOURS.items():
        if built_sha(os.path.join(d, so)) != want:
            subprocess.check_call(["make", "-s", "-j8", "-C", d] + args)
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def topo_paths(tmp_path_factory):
    """Decompressed bundled topologies (the reference installs them decompressed,
    resource/CMakeLists.txt:3-22)."""
    import lzma
    d = tmp_path_factory.mktemp("topologies")
    out = {}
    for name, fn in {"simple": "topology.simple.graphml.xml.xz", "full": "topology.graphml.xml.xz",
                     "plab": "topology.plab.graphml.xml.xz"}.items():
        p = d / fn[:-3]
        p.write_bytes(lzma.open(os.path.join(GOLDEN, "topologies", fn)).read())
        out[name] = str(p)
    return out


def gpu_available() -> bool:
    try:
        from shadow_amd import routes
        return routes.device_count() > 0
    except Exception:
        return False
