#!/usr/bin/env python3
"""Phase breakdown of k_routes_sssp with the diagnostic build
(SHDR_LIB_VARIANT=diag; make -C shadow_amd diag). Prints per-phase share of
workgroup wall ticks (100 MHz realtime counter) and work counters."""
import ctypes as C
import os
import sys
import time

os.environ["SHDR_LIB_VARIANT"] = "diag"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from shadow_amd import _lib  # noqa: E402
from shadow_amd.routes import SHDR_TIMING, Engine, Graph  # noqa: E402

NAMES = ["t_init", "t_relax", "t_phase1", "t_pred", "t_epilogue", "rounds", "drains", "scan_vertices", "items",
         "arcs", "atomics", "improvements", "walk_steps", "buckets", "improve_events", "drain_rows", "t_drain", "active_lane_items"]


def run(g, src, dst, delta=None, label="", variant=None):
    lib = _lib.load()
    eng = Engine(g)
    if delta:
        eng.set_delta(delta)
    if variant is not None:
        eng.set_variant(variant)
    buf = (C.c_ulonglong * 32)()
    eng.compute(src[:64], dst)  # warm
    # pass 1 issues buckets by landmark spread, later passes by measured duration
    for _ in range(int(os.environ.get("DIAG_PASSES", "1")) - 1):
        eng.compute(src, dst)
    lib.shdr_diag_read(buf, 32, 1)
    t0 = time.perf_counter()
    eng.compute(src, dst, flags=SHDR_TIMING)
    wall = time.perf_counter() - t0
    lib.shdr_diag_read(buf, 32, 1)
    d = dict(zip(NAMES, list(buf)[:len(NAMES)]))
    tt = d["t_init"] + d["t_relax"] + d["t_pred"] + d["t_epilogue"]
    print(f"== {label} variant={variant} S={len(src)} T={len(dst)} delta={delta} kernel {eng.timing()} wall {wall*1e3:.1f} ms")
    for k in ["t_init", "t_relax", "t_phase1", "t_drain", "t_pred", "t_epilogue"]:
        print(f"   {k:12s} {d[k] / 1e2 / max(d['buckets'], 1):10.1f} us/bucket  {100.0 * d[k] / max(tt, 1):5.1f}%")
    A = g.E * 2
    nb = max(d["buckets"], 1)
    for k in ["rounds", "drains", "scan_vertices", "items", "arcs", "atomics", "improvements", "walk_steps",
              "improve_events", "drain_rows", "active_lane_items"]:
        print(f"   {k:14s} {d[k] / nb:14.1f} per bucket")
    gd = list(buf)
    if gd[24]:
        start = (~gd[23]) & (2**64 - 1)
        mx, mn, mean = gd[21] - start, ((~gd[22]) & (2**64 - 1)) - start, gd[20] / gd[24] - start
        print(f"   main launch: {gd[24]} workgroups exit between {mn / 100:.0f} and {mx / 100:.0f} us (mean {mean / 100:.0f} us)")
    if hasattr(lib, "shdr_diag_buckets"):
        st, du = (C.c_ulonglong * 8192)(), (C.c_ulonglong * 8192)()
        lib.shdr_diag_buckets(st, du, 8192)
        du = np.array(du[:]); st = np.array(st[:])
        nbt = int((du > 0).sum())
        if nbt:
            bd = du[:nbt] / 100.0  # us
            s0 = st[:nbt] - st[:nbt].min()
            q = np.percentile(bd, [0, 10, 50, 90, 100])
            print("   bucket us: min %.0f p10 %.0f p50 %.0f p90 %.0f max %.0f; cv %.3f" % (*q, bd.std() / bd.mean()))
            print("   bucket end (us) max %.0f; sum/256 %.0f" % ((s0 / 100.0 + bd).max(), bd.sum() / 256))
            np.save(os.path.join("gpurun_out", f"buckets_{label}.npy"), np.stack([s0 / 100.0, bd]))
            order = (C.c_int32 * len(src))()
            lib.shdr_diag_order(C.c_void_p(eng._h), order, len(src))
            np.save(os.path.join("gpurun_out", f"order_{label}.npy"), np.array(order[:]))
    # per-degree counters (routes.hip DIAG slots 18, 19, 25)
    A_real = A
    print(f"   head_rows      {gd[18] / nb:14.1f} per bucket ({gd[18] / nb / A_real:.3f} A)")
    print(f"   hub_rows       {gd[19] / nb:14.1f} per bucket (vertices of degree >= 64: "
          f"{gd[19] / max(gd[18], 1):.3f} of the head rows)")
    hubs = int(os.environ.get("DIAG_HUBS", "0")) or None
    print(f"   hub_expansions {gd[25] / nb:14.1f} per bucket" +
          (f" ({gd[25] / nb / hubs:.2f} per hub)" if hubs else ""))
    if gd[26]:
        print(f"   cluster barriers {gd[26] / nb:10.1f} per member-bucket, {gd[27] / 1e2 / max(gd[26], 1):.2f} us each "
              f"(lane 0 arrive to acquire; {100.0 * gd[27] / max(tt, 1):.1f}% of member ticks)")
    print(f"   active lanes per item {d['active_lane_items'] / max(d['items'], 1):.2f}")
    print(f"   arcs/A per bucket {d['arcs'] / nb / A:.2f}; scan/V per bucket {d['scan_vertices'] / nb / g.V:.2f}")


if __name__ == "__main__":
    import bench
    wl = sys.argv[2] if len(sys.argv) > 2 else "cfg4"
    g, hosts, _, _ = bench.make_workload(wl)
    vs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,4").split(",")]
    src = hosts
    parts = [(wl, src)]
    if os.environ.get("PART"):  # strong-scaling shard: part PART_IDX (or every part: all) of Engine.partition
        n = int(os.environ["PART"])
        part = Engine(g).partition(hosts, n)
        which = os.environ.get("PART_IDX", "0")
        idx = range(n) if which == "all" else [int(which)]
        parts = [(f"{wl}_p{n}_{i}", hosts[part == i]) for i in idx]
    ef, et, _, _, _ = g.export()
    keep = ef != et
    deg = np.bincount(np.concatenate([ef[keep], et[keep]]), minlength=g.V)
    os.environ["DIAG_HUBS"] = str(int((deg >= 64).sum()))
    for label, src in parts:
        for var in vs:
            run(g, src, hosts, label=label, variant=var)
