import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def _lib_is_stale() -> bool:
    """The product library's compiled-in routes.hip sha (shdr_version) differs from
    the tree's routes.hip. Checked in a child process, so this process loads the
    library only after any rebuild."""
    code = ("from shadow_amd.routes import lib_kernel_sha, src_kernel_sha; "
            "import sys; sys.exit(0 if lib_kernel_sha() == src_kernel_sha() else 3)")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True)
    return r.returncode != 0


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    # build the in-tree libraries if a fresh checkout lacks them or the product
    # library was compiled from another routes.hip than the tree's (CPU-only step)
    if not os.path.exists(os.path.join(ROOT, "shadow_amd", "libshdtopology.so")) or _lib_is_stale():
        subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(ROOT, "shadow_amd"), "all", "bchk"])
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
