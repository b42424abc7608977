"""Schedule-only engine knobs never change results, through the
experiments flavour that compiles them (SHDR_EXPERIMENTS); the cases run in a fresh
process because one process loads one library flavour (shadow_amd/_lib.py)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(900)
def test_schedule_knobs_never_change_results():
    lib = os.path.join(ROOT, "shadow_amd", "libshdtopology_exp.so")
    from tests.conftest import built_sha, tree_sha
    assert built_sha(lib) == tree_sha(), (built_sha(lib), tree_sha(), ("build it first: make -C shadow_amd flavor NAME=exp DEFS=-DSHDR_EXPERIMENTS "
                                 "(__graft_entry__.build does)"))
    env = dict(os.environ, SHDR_LIB_VARIANT="exp")
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "exp_knob_cases.py")], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=600)
    print(r.stdout[-4000:], r.stderr[-4000:])
    assert r.returncode == 0, r.stderr[-4000:]
    assert "exp knob cases: 18 passed" in r.stdout
