#!/usr/bin/env python3
"""Share of the relaxation's head-row accesses that go to pendant vertices (experiments only).

A pendant vertex (every arc joins one single neighbour) never enters a pending set
(DESIGN.md §3.1), but the arc from its neighbour is still relaxed, reading its row, every
time the neighbour is expanded. Weighting each arc by its tail's expansions per bucket
(3.77 for degree >= 64; 1.1 otherwise) estimates what dropping those arcs
from the arc blocks could save. usage: python tools/pendant_share.py [cfg5|cfg4]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "cfg5"
    g, _, _, _ = bench.make_workload(wl)
    ef, et, _, _, _ = g.export()
    keep = ef != et
    ef, et = ef[keep].astype(np.int64), et[keep].astype(np.int64)
    V = g.V
    src = np.concatenate([ef, et])
    dst = np.concatenate([et, ef])
    deg = np.bincount(src, minlength=V)
    order = np.lexsort((dst, src))
    s2, d2 = src[order], dst[order]
    first_pair = np.r_[True, (s2[1:] != s2[:-1]) | (d2[1:] != d2[:-1])]
    neighbours = np.bincount(s2[first_pair], minlength=V)
    pend = neighbours == 1
    into_pend = pend[dst] & ~pend[src]
    exp = np.where(deg >= 64, 3.77, 1.1)
    share = (exp[src] * into_pend).sum() / (exp[src] * ~pend[src]).sum()
    blk_now = np.ceil(deg / 8.0)
    blk_new = np.ceil((deg - np.bincount(src[into_pend], minlength=V)) / 8.0)
    w = exp * ~pend
    print(f"{wl}: V {V}, pendant vertices {int(pend.sum())} ({pend.mean():.3f}), arcs into them "
          f"{int(into_pend.sum())} ({into_pend.mean():.3f} of arcs)")
    print(f"expansion-weighted share of head-row accesses to pendant heads: {share:.3f}")
    print(f"expansion-weighted arc blocks: {(w * blk_now).sum():.3e} -> {(w * blk_new).sum():.3e} without them")


if __name__ == "__main__":
    main()
