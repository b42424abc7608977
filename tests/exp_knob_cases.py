"""Schedule-only knobs of the experiments flavour (libshdtopology_exp.so, built with
-DSHDR_EXPERIMENTS by `make -C shadow_amd flavor NAME=exp DEFS=-DSHDR_EXPERIMENTS`),
run by tests/test_gpu_exp_knobs.py in a fresh process with SHDR_LIB_VARIANT=exp
(one library flavour per process).

Knobs that only change the schedule: far-set marking
(SHDR_FAR_SKIP 0 / 2 / 3: always, lane-local rule, skip inside clusters too), hub
lag (SHDR_HUB_LAG), the arena base alignment, the landmark count and the window
rule, the per-bucket fill of the distance rows (SHDR_NOFILL=0 restores it), with the far set in slot bytes (pending mode 1, as on cfg5) and in LDS (mode
2). Every setting must give the oracle's tables bit for bit, also when every vertex
is a source (slots run many buckets, so pending state left over from one bucket
would show in the next). The product library compiles none of these branches.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from oracle import py_oracle as po  # noqa: E402
from shadow_amd import _lib  # noqa: E402
from shadow_amd.routes import Engine, Graph, lib_kernel_sha, src_kernel_sha  # noqa: E402
from tests.util import bits  # noqa: E402

KNOBS = [{"SHDR_FAR_SKIP": "0"}, {"SHDR_FAR_SKIP": "2"}, {"SHDR_HUB_LAG": "2"},
         {"SHDR_HUB_LAG": "8", "SHDR_FAR_SKIP": "2"}, {"SHDR_ARENA_ALIGN_MB": "64"},
         {"SHDR_LANDMARKS": "2"}, {"SHDR_LANDMARKS": "8"}, {"SHDR_DELTA_RULE": "0"},
         {"SHDR_NOFILL": "0"}]
ALL = sorted({k for d in KNOBS for k in d})


def main() -> int:
    assert _lib.LIB_PATH.endswith("libshdtopology_exp.so"), _lib.LIB_PATH
    # the flavour was built from the tree's sources (tests/conftest.py rebuilds stale flavours)
    assert lib_kernel_sha() == src_kernel_sha(), (lib_kernel_sha(), src_kernel_sha())
    g = Graph.generate("chunglu", 7000, 3, 31)
    src = np.random.default_rng(6).choice(g.V, 400, replace=False).astype(np.int32)
    allv = np.arange(g.V, dtype=np.int32)
    dst = np.arange(0, g.V, 17, dtype=np.int32)
    og = po.OracleGraph.from_graph(g)
    ref = og.routes(src, dst, po.MODE_CANONICAL, threads=8)
    ref_all = og.routes(allv, dst, po.MODE_CANONICAL, threads=8)
    n = 0
    for mode in ("1", "2"):
        os.environ["SHDR_PENDING_LDS"] = mode
        os.environ["SHDR_CLUSTER"] = "1"
        for knobs in KNOBS:
            for k in ALL:
                os.environ.pop(k, None)
            os.environ.update(knobs)
            eng = Engine(g)
            t = eng.compute(src, dst, hops=True)
            lat, rel, hops, rmin = ref
            assert np.array_equal(bits(t.lat), bits(lat)), (mode, knobs)
            assert np.array_equal(bits(t.rel), bits(rel)), (mode, knobs)
            assert np.array_equal(t.hops, hops), (mode, knobs)
            assert np.array_equal(bits(t.row_min), bits(rmin)), (mode, knobs)
            t2 = eng.compute(allv, dst)
            assert np.array_equal(bits(t2.lat), bits(ref_all[0])), (mode, knobs)
            assert np.array_equal(bits(t2.rel), bits(ref_all[1])), (mode, knobs)
            del eng
            n += 1
            print(f"exp knobs ok: mode {mode} {knobs}", flush=True)
    print(f"exp knob cases: {n} passed", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
