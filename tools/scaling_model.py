#!/usr/bin/env python3
"""Wave model of a strong-scaling shard (CPU only): which bucket layouts could take
cfg5 over N GPUs to a given efficiency (round-5 verdict item 4).

Every GPU has `slots` resident workgroups (256 CUs, one 1024-thread workgroup
each). A K=16 bucket takes t16 = 1 whatever its fill (its rounds are set by the
graph), a K=8 bucket t8 = R8 * t16 (measured 0.79 on cfg5), and a bucket shared
by a cluster of cl workgroups t16 / (E * cl) (E = per-CU efficiency of the
cluster, measured 0.68-0.77; PM 1 clusters, the only kind cfg5's 1e6 vertices
allow, are gated off). Buckets run in whole waves of the resident
slots, and a launch ends with its slowest slot (the dynamic queue packs buckets;
per-CU work is integral). The full table's time over one GPU is the same model's
best layout for S = 50,000; efficiency(N) = T(S) / (N * T(S / N)).

Layouts per shard of S rows:
  plain        ceil(S/16) K16 buckets over `slots`
  tail         full K16 waves, the partial last wave (<= slots/2 buckets) as K8 buckets
  balanced     S <= 8 * slots: K8 buckets of S/slots rows
  cluster cl   ceil(S/16) buckets over slots/cl clusters
  mixed cl     full K16 waves, the partial last wave as cl-wide clusters
               (needs the clusters co-resident as the plain workgroups exit)
Also: the smallest cluster efficiency E that reaches a target efficiency at N.
usage: python tools/scaling_model.py [--target 0.86] [--r8 0.79] [--e 0.7]
"""
import argparse
import math


def layouts(S, slots, r8, e, cmax=4):
    out = {}
    nb = math.ceil(S / 16)
    out["plain"] = math.ceil(nb / slots)
    waves, rem = divmod(nb, slots)
    if waves >= 1 and 0 < rem <= slots // 2:
        # half-width buckets of the last wave's rows fill the CUs as they free
        out["tail"] = waves + r8 * math.ceil(2 * rem / slots)
    if S <= 8 * slots:
        out["balanced"] = r8 * 1.0  # one wave of <= 8-row buckets (a bucket costs ~the same at any fill)
    for cl in range(2, cmax + 1):
        cs = slots // cl
        out[f"cluster{cl}"] = math.ceil(nb / cs) / (e * cl)
        if waves >= 1 and rem > 0:
            out[f"mixed{cl}"] = waves + math.ceil(rem / cs) / (e * cl)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--target", type=float, default=0.86)
    ap.add_argument("--r8", type=float, default=0.79)
    ap.add_argument("--e", type=float, default=0.70)
    ap.add_argument("--slots", type=int, default=256)
    ap.add_argument("--S", type=int, default=50_000)
    a = ap.parse_args()
    full = layouts(a.S, a.slots, a.r8, a.e)
    tfull = min(full["plain"], full.get("tail", 1e9))  # the full table runs plain buckets (+ tail)
    print(f"# S = {a.S}, {a.slots} slots, K8 bucket = {a.r8} K16 bucket, cluster per-CU efficiency {a.e}")
    print(f"# full table: {tfull:.2f} bucket times ({ {k: round(v, 2) for k, v in full.items() if k in ('plain', 'tail')} })")
    for N in (2, 4, 8):
        S = math.ceil(a.S / N)
        ls = layouts(S, a.slots, a.r8, a.e)
        best = min(ls, key=ls.get)
        eff = {k: tfull / (N * v) for k, v in ls.items()}
        print(f"N = {N}: shard {S} rows ({math.ceil(S / 16)} K16 buckets, {math.ceil(S / 16) / a.slots:.2f} waves); "
              f"best {best} {ls[best]:.2f} -> efficiency {eff[best]:.3f}")
        print("   " + ", ".join(f"{k} {v:.2f} ({eff[k]:.2f})" for k, v in sorted(ls.items(), key=lambda x: x[1])))
        # the cluster efficiency a clustered layout would need for the target
        need = {}
        for k in ls:
            if not (k.startswith("cluster") or k.startswith("mixed")):
                continue
            lo, hi = 0.3, 1.0
            if tfull / (N * layouts(S, a.slots, a.r8, hi)[k]) < a.target:
                need[k] = None
                continue
            for _ in range(40):
                mid = (lo + hi) / 2
                if tfull / (N * layouts(S, a.slots, a.r8, mid)[k]) >= a.target:
                    hi = mid
                else:
                    lo = mid
            need[k] = hi
        print(f"   cluster efficiency E needed for {a.target}: " +
              ", ".join(f"{k} {'unreachable' if v is None else f'{v:.2f}'}" for k, v in need.items()))


if __name__ == "__main__":
    main()
