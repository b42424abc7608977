"""The whole BASELINE tables at the relaxation's fixed point, through the verify
flavour (SHDR_VERIFY): cfg4's full table and its 8 strong-scaling shards (3-wide
clusters), and cfg5's full 50,000 x 50,000 table, every lane of every vertex checked
on the device (tests/verify_full_cases.py). The cases run in a fresh process because
one process loads one library flavour (shadow_amd/_lib.py, SHDR_LIB_VARIANT)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(900)
def test_baseline_tables_at_relaxation_fixed_point():
    from tests.conftest import built_sha, tree_sha
    lib = os.path.join(ROOT, "shadow_amd", "libshdtopology_verify.so")
    assert built_sha(lib) == tree_sha(), (built_sha(lib), tree_sha(), "build it first: make -C shadow_amd flavor "
                                          "NAME=verify DEFS=-DSHDR_VERIFY (__graft_entry__.build does)")
    env = dict(os.environ, SHDR_LIB_VARIANT="verify")
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "verify_full_cases.py")], env=env,
                       cwd=ROOT, capture_output=True, text=True, timeout=800)
    print(r.stdout[-6000:], r.stderr[-4000:])
    assert r.returncode == 0, r.stderr[-4000:]
    assert "verify full cases: 10 passed" in r.stdout
