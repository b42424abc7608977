#!/usr/bin/env python3
"""Round-5 analysis of the PM 1 cluster fault (experiments only, not product code).

Reads the dump written by the round-4 tree's host-side patch
(profiles/r05_pm1_dump_host_patch.diff, SHDR_DUMP=<file>) after the failing launch
of tools/repro_pm1.py (Chung-Lu 7,000 vertices seed 8, 300 sources, every 11th
vertex a target, 4-wide PM 1 clusters), and checks it against the oracle:
  1. distances of the dumped slots vs the oracle's Dijkstra, bit for bit;
  2. predecessor entries on the targets' chains vs the oracle's canonical tree;
  3. which chain-pass level the missing entries belong to, and whether they
     follow the member that owns or marks them.
usage: python tools/pm1_dump_analysis.py gpurun_out/pm1_dump2.bin
"""
import os
import sys
from collections import Counter

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import py_oracle as po  # noqa: E402
from shadow_amd.routes import Graph  # noqa: E402


def load(path):
    b = open(path, "rb").read()
    o = 0

    def take(dt, n):
        nonlocal o
        a = np.frombuffer(b, dt, n, o)
        o += a.nbytes
        return a

    S, T, _, ng, V, kE = (int(x) for x in take(np.int32, 6))
    d = {"S": S, "T": T, "V": V, "rec": take(np.int32, kE)}
    d["src"] = take(np.int32, S)
    d["rowmap"] = take(np.int32, S)
    d["boff"] = take(np.int32, ng + 1)
    d["soff"] = take(np.float64, S)
    d["lat"] = take(np.float64, S * T).reshape(S, T)
    d["hops"] = take(np.int32, S * T).reshape(S, T)
    d["newid"] = take(np.int32, V)
    stride, off_pred, K, nsl = (int(x) for x in take(np.int64, 4))
    d.update(stride=stride, off_pred=off_pred, K=K, nsl=nsl)
    d["arena"] = np.frombuffer(b, np.uint8, nsl * stride, o)
    return d


def main():
    d = load(sys.argv[1])
    V, K, stride, off_pred = d["V"], d["K"], d["stride"], d["off_pred"]
    g = Graph.generate("chunglu", 7000, 3, 8)
    og = po.OracleGraph.from_graph(g)
    newid = d["newid"].astype(np.int64)
    oldid = np.empty(V, np.int64)
    oldid[newid] = np.arange(V)
    tdev = newid[np.arange(0, g.V, 11)]
    print("guard record:", d["rec"][:16].tolist())
    src0 = np.random.default_rng(4).choice(g.V, 300, replace=False).astype(np.int32)
    lat, _, _, _ = og.routes(src0, np.arange(0, g.V, 11, dtype=np.int32), po.MODE_CANONICAL, threads=8)
    nan_rows = int(np.isnan(d["lat"]).all(axis=1).sum())
    bad = d["lat"].view(np.uint64) != lat.view(np.uint64)
    print(f"table: {int(bad.sum())} of {bad.size} latencies differ from the oracle "
          f"(all NaN: {int((bad & np.isnan(d['lat'])).sum())}); rows entirely NaN: {nan_rows}")
    dist_ok = dist_n = 0
    lvl_need, lvl_miss = Counter(), Counter()
    owner_need, owner_miss = Counter(), Counter()
    miss_sets = []
    for sl in range(d["nsl"]):
        base = sl * stride
        dist = d["arena"][base: base + V * K * 8].view(np.float64).reshape(V, K)
        pred = d["arena"][base + off_pred: base + off_pred + V * K * 8].view(np.int32).reshape(V, K, 2)
        lanes = [ln for ln in range(K) if (dist[:, ln] == 0.0).any()]
        trees = {}
        for ln in lanes:
            z = int(np.where(dist[:, ln] == 0.0)[0][0])
            dd, _ = og.dijkstra(int(oldid[z]))
            dist_n += 1
            dist_ok += np.array_equal(dist[newid, ln].view(np.uint64), dd.view(np.uint64))
            op, _ = og.canonical_pred(int(oldid[z]), dd)
            pdev = np.full(V, -1)
            m = op >= 0
            pdev[newid[np.where(m)[0]]] = newid[op[m]]
            trees[ln] = (z, pdev)
        # chain-pass levels as the kernel builds them (any lane), device numbering
        level = np.full(V, -1)
        level[tdev] = 0
        cur, lv, markers = set(tdev.tolist()), 0, {}
        while cur:
            nxt = set()
            for x in cur:
                for ln in lanes:
                    z, pdev = trees[ln]
                    p = pdev[x]
                    if x == z or p < 0:
                        continue
                    if level[p] < 0 or p in nxt:
                        markers.setdefault(p, set()).add(x)
                        if level[p] < 0:
                            level[p] = lv + 1
                            nxt.add(p)
            cur, lv = nxt, lv + 1
        miss = set()
        for u in np.where(level >= 0)[0]:
            if any(u == trees[ln][0] for ln in lanes):
                continue
            ok = all(pred[u, ln, 0] == trees[ln][1][u] for ln in lanes if trees[ln][1][u] >= 0)
            lvl_need[int(level[u])] += 1
            owner_need[int((u >> 5) % 4)] += 1
            if not ok:
                lvl_miss[int(level[u])] += 1
                owner_miss[int((u >> 5) % 4)] += 1
                miss.add(int(u))
        miss_sets.append(miss)
    print(f"distances: {dist_ok} of {dist_n} dumped source lanes bit-exact vs the oracle's Dijkstra")
    print("chain-pass entries needed / wrong by level:",
          {k: (lvl_need[k], lvl_miss[k]) for k in sorted(lvl_need)})
    print("needed / wrong by owning member (word % 4):",
          {k: (owner_need[k], owner_miss[k]) for k in sorted(owner_need)})
    common = set.intersection(*miss_sets) if miss_sets else set()
    union = set.union(*miss_sets) if miss_sets else set()
    print(f"missing vertices: {len(union)} over the dumped slots, {len(common)} missing in every slot")


if __name__ == "__main__":
    main()
