"""Cluster mode through the bounds-checked flavour (SHDR_BCHK), deterministically.

Cluster mode's cross-workgroup barriers once published chain-pass marks before
they landed (wrong paths with equal latencies under some timings; round 2,
commit 1d88a84). The timing-dependent parity tests (test_cluster_buckets) may
miss such a race; the bounds-checked flavour poisons every predecessor entry at
bucket start, so a walk over an entry the pass never wrote trips guard 32 on
every run. The cases run in a fresh process because one process loads one
library flavour (shadow_amd/_lib.py, SHDR_LIB_VARIANT).
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(900)
def test_cluster_cases_bounds_checked():
    lib = os.path.join(ROOT, "shadow_amd", "libshdtopology_bchk.so")
    from tests.conftest import built_sha, tree_sha
    assert built_sha(lib) == tree_sha(), (built_sha(lib), tree_sha(), "build it first: make -C shadow_amd bchk (__graft_entry__.build does)")
    env = dict(os.environ, SHDR_LIB_VARIANT="bchk")
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "bchk_cluster_cases.py")], env=env,
                       cwd=ROOT, capture_output=True, text=True, timeout=600)
    print(r.stdout[-4000:], r.stderr[-4000:])
    assert r.returncode == 0, r.stderr[-4000:]
    assert "bchk cluster cases: 12 passed" in r.stdout
