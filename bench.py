#!/usr/bin/env python3
"""Benchmark: all-sources latency+reliability route tables on MI355X.

One "step" = one pass of the hot path over one batch: every source row of this
rank x every attached target (shortest path + ordered latency/reliability
epilogue + row minima, one kernel launch), then the scheduler-window exchange
(RCCL all-reduce(MIN) of the global minimum path latency) across ranks.
Inputs (graph CSR, source/target lists) are resident in HBM before timing.

Scaling (default "weak"): every rank routes the same number of source rows
(the workload's host count) to the same attached targets, so per-GPU work is
fixed and N=1 is exactly the BASELINE config.  Rank r's sources are the r-th
block of a seeded vertex permutation whose first block is the attached host
set.  With --scaling strong the host set is split over the ranks instead.
The all-gather of the row shards (every rank receiving the whole table over
xGMI) is timed separately after the timed steps and reported as
"allgather_ms" (report gather time separately).

Workloads (BASELINE.json configs; synthetic data):
  cfg4 (default) synthetic Barabasi-Albert n=100,000 m=3 seed 1, 10,000 hosts
                 -> 1e8 source-paths per rank per step
  cfg5           synthetic Chung-Lu power law n=1,000,000, 50,000 hosts
  cfg2 / cfg3    bundled full / PlanetLab topology, all vertices (direct edge)

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg4]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import lzma
import os
import sys
import tempfile
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from shadow_amd.routes import SHDR_TIMING, Engine, Graph  # noqa: E402
from shadow_amd.shard import allgather_rows, allreduce_min, local_min, shard_rows  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)


def make_workload(name: str):
    """-> (graph, hosts[int32] (attached targets), vertex pool for extra weak-scaling sources, description)"""
    if name in ("cfg4", "cfg5"):
        if name == "cfg4":
            g = Graph.generate("ba", 100_000, 3, 1)
            nh = 10_000
            desc = "cfg4: synthetic Barabasi-Albert n=100000 m=3 seed=1, 10000 attached hosts"
        else:
            g = Graph.generate("chunglu", 1_000_000, 3, 1)
            nh = 50_000
            desc = "cfg5: synthetic Chung-Lu power law n=1000000 mean degree ~6 seed=1, 50000 attached hosts"
        pool = np.random.default_rng(1).permutation(g.V).astype(np.int32)
        hosts = np.sort(pool[:nh])
    elif name in ("cfg2", "cfg3"):
        fn = {"cfg2": "topology.graphml.xml.xz", "cfg3": "topology.plab.graphml.xml.xz"}[name]
        raw = lzma.open(os.path.join(ROOT, "tests", "golden", "topologies", fn)).read()
        with tempfile.NamedTemporaryFile(suffix=".graphml.xml", delete=False) as f:
            f.write(raw)
            path = f.name
        g = Graph.load_graphml(path)
        os.unlink(path)
        hosts = np.arange(g.V, dtype=np.int32)
        pool = hosts
        desc = f"{name}: bundled {fn[:-3]}, one host per vertex (complete graph: direct edge)"
    else:
        raise SystemExit(f"unknown workload {name}")
    return g, hosts, pool, {"workload": desc}


def rank_sources(hosts, pool, world, rank, scaling):
    """-> (rows padded, n_real): this rank's source rows."""
    if scaling == "strong":
        rows, n_real, _ = shard_rows(hosts, world, rank)
        return rows, n_real
    S = len(hosts)
    if rank == 0:
        return hosts, S
    if (rank + 1) * S <= len(pool):
        return np.sort(pool[rank * S:(rank + 1) * S]), S
    # not enough distinct vertices for a disjoint block: cycle through the pool
    idx = (np.arange(S) + rank * S) % len(pool)
    return np.sort(pool[idx]), S


def cpu_baseline(g: Graph, hosts: np.ndarray, complete: bool, budget_s: float = 15.0) -> dict:
    """Reference-faithful CPU path (oracle restatement of igraph Dijkstra + the
    epilogue, or the direct edge) on ONE core, on a bounded sample of sources."""
    from oracle import py_oracle as po  # test infrastructure: the baseline, never the measured path

    og = po.OracleGraph.from_graph(g)
    mode = po.MODE_COMPLETE if complete else po.MODE_IGRAPH
    T = len(hosts)
    n = min(4, len(hosts))
    t0 = time.perf_counter()
    og.routes(hosts[:n], hosts, mode, threads=1)
    dt = time.perf_counter() - t0
    n2 = int(min(len(hosts), max(n, budget_s / max(dt / n, 1e-9))))
    if n2 > n:
        t0 = time.perf_counter()
        og.routes(hosts[:n2], hosts, mode, threads=1)
        dt = time.perf_counter() - t0
        n = n2
    out = {"value": n * T / dt, "unit": "source-paths/s", "cores": 1, "kind": "port",
           "sample": f"{n} of {len(hosts)} sources x {T} targets, {dt:.1f} s on 1 core "
                     f"({'direct edge' if complete else 'binary-heap Dijkstra + ordered epilogue'}); "
                     "extrapolation: sources are independent"}
    # upper bound: the same port, source-parallel over this process's CPU share
    cores = max(1, min(16, len(os.sched_getaffinity(0))))
    if cores > 1 and not complete:
        m = int(min(len(hosts), max(cores, n * cores * 0.3)))  # ~0.3 x the 1-core budget of wall time
        t0 = time.perf_counter()
        og.routes(hosts[:m], hosts, mode, threads=cores)
        dt2 = time.perf_counter() - t0
        out["all_cores"] = {"value": m * T / dt2, "cores": cores,
                            "sample": f"{m} sources x {T} targets, {dt2:.1f} s on {cores} threads"}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default=os.environ.get("SHDR_BENCH_WORKLOAD", "cfg4"))
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true", help="skip the (separately timed) all-gather")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL; gloo only "
                    "to rehearse the multi-rank flow with every rank on one GPU, --same-device)")
    ap.add_argument("--same-device", action="store_true", help="every rank uses cuda:0 (rehearsal)")
    ap.add_argument("--no-side-configs", action="store_true", help="skip the bundled-topology side lines")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)

    g, hosts, pool, desc = make_workload(args.workload)
    info = g.check()
    complete = bool(info.is_complete)
    T = len(hosts)
    mine, n_real = rank_sources(hosts, pool, world, rank, args.scaling)
    per = len(mine)
    S_total = T * world if args.scaling == "weak" else T
    eng = Engine(g, device=local)
    lat = torch.empty((per, T), dtype=torch.float64, device=dev)
    rel = torch.empty((per, T), dtype=torch.float64, device=dev)
    rmin = torch.empty((per,), dtype=torch.float64, device=dev)
    gmin = torch.empty((1,), dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)
    kernel_ms = []  # per step: {kernel name: ms} (HIP events on the launch stream)

    def step(record: bool):
        eng.compute_device(mine, hosts, lat.data_ptr(), rel.data_ptr(), rmin.data_ptr(), None, flags=SHDR_TIMING,
                           stream=stream.cuda_stream)
        if record:
            kernel_ms.append(eng.timing())
        gmin.copy_(allreduce_min(local_min(rmin, n_real)))

    for _ in range(args.warmup):
        step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    gather = None
    if world > 1 and not args.no_gather:
        # the table exchange: every rank receives every row shard (RCCL all-gather over xGMI)
        lat_all = torch.empty((per * world, T), dtype=torch.float64, device=dev)
        rel_all = torch.empty((per * world, T), dtype=torch.float64, device=dev)
        allgather_rows(lat, lat_all)
        allgather_rows(rel, rel_all)
        dist.barrier()
        torch.cuda.synchronize(dev)
        tg = time.perf_counter()
        allgather_rows(lat, lat_all)
        allgather_rows(rel, rel_all)
        torch.cuda.synchronize(dev)
        dist.barrier()
        tgm = torch.tensor([time.perf_counter() - tg], dtype=torch.float64, device=dev)
        dist.all_reduce(tgm, op=dist.ReduceOp.MAX)
        gbytes = 2 * lat_all.numel() * 8
        gather = {"allgather_ms": float(tgm.item()) * 1e3, "table_bytes_per_rank": gbytes,
                  "value_incl_gather": S_total * T / (elapsed / args.steps + float(tgm.item()))}
        del lat_all, rel_all

    V = info.vertex_count
    A = int(eng_arcs(g))
    names = sorted({k for d in kernel_ms for k in d if k != "routes_pass"})
    per_kernel = {k: float(np.mean([d.get(k, 0.0) for d in kernel_ms])) for k in names}
    # One table pass = the main launch (+ a half-width tail launch when the last of >= 2
    # full waves of buckets would be at most half full, running concurrently on a second stream, routes.hip):
    # bytes and time are taken over the pass, fork to join (HIP events).
    passes = [d["routes_pass"] for d in kernel_ms if "routes_pass" in d]
    k_ms = float(np.mean(passes)) if passes else (sum(per_kernel.values()) if per_kernel else float("nan"))
    if complete:
        bytes_per_launch = 32.0 * per * T  # lat+loss read, lat+rel written per pair
    else:
        bytes_per_launch = per * (12.0 * A + 20.0 * V) + 16.0 * per * T
    kname = " + ".join(names)
    achieved = bytes_per_launch / (k_ms * 1e-3) / 1e9
    traffic = load_pmc_traffic(args.workload, names, per)
    result = {
        "metric": "source-paths/sec (all-sources latency+reliability)",
        "value": S_total * T * args.steps / elapsed,
        "unit": "source-paths/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic" if args.workload in ("cfg4", "cfg5") else "reference bundled topology",
        "config": dict(desc, V=V, arcs=A, sources=S_total, targets=T, sources_per_rank=per,
                       parallelism=f"source-shard x{world}" + (
                           f" + {'RCCL' if args.backend == 'nccl' else args.backend} all-reduce(MIN)" if world > 1 else ""),
                       branch="direct-edge" if complete else "shortest-path"),
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": kname,
                     "kernel_ms": k_ms, "kernel_ms_each": per_kernel,
                     "kernel_ms_note": ("kernel_ms = one table pass = one launch (HIP events on its stream)"
                                        if len(names) == 1 else
                                        "kernel_ms = one table pass, fork to join; the tail launch overlaps the main "
                                        "launch (its time is counted from the fork)"),
                     "algorithmic_bytes_per_launch": bytes_per_launch},
        "global_min_latency_ms": float(gmin.item()),
    }
    if gather:
        result["allgather"] = gather
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(g, hosts, complete)
    if rank == 0 and world == 1 and args.workload == "cfg4" and not args.no_side_configs:
        result["side_configs"] = side_configs(local)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def side_configs(device: int) -> dict:
    """BASELINE configs 2 and 3 (the reference's bundled full and PlanetLab topologies,
    one host per vertex). Both are complete graphs, so the reference answers every
    pair from the direct edge: a small dense gather, timed here for the
    record next to the headline shortest-path workload."""
    out = {}
    for name in ("cfg2", "cfg3"):
        g, hosts, _, desc = make_workload(name)
        eng = Engine(g, device=device)
        T = len(hosts)
        dev = torch.device("cuda", device)
        lat = torch.empty((T, T), dtype=torch.float64, device=dev)
        rel = torch.empty((T, T), dtype=torch.float64, device=dev)
        rmin = torch.empty((T,), dtype=torch.float64, device=dev)
        st = torch.cuda.current_stream(dev).cuda_stream
        for _ in range(3):
            eng.compute_device(hosts, hosts, lat.data_ptr(), rel.data_ptr(), rmin.data_ptr(), None, stream=st)
        torch.cuda.synchronize(dev)
        reps = 50
        t0 = time.perf_counter()
        for _ in range(reps):
            eng.compute_device(hosts, hosts, lat.data_ptr(), rel.data_ptr(), rmin.data_ptr(), None, flags=SHDR_TIMING,
                               stream=st)
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / reps
        kms = eng.timing().get("k_routes_direct", float("nan"))
        out[name] = {"workload": desc["workload"], "pairs": T * T, "value": T * T / dt, "unit": "source-paths/s",
                     "ms_per_table": dt * 1e3, "kernel_ms": kms,
                     "note": "complete graph: direct-edge branch; launch-latency bound at this size"}
    return out


def eng_arcs(g: Graph) -> int:
    ef, et, _, _, _ = g.export()
    loops = int((ef == et).sum())
    return (len(ef) - loops) * (1 if g.directed else 2)


def load_pmc_traffic(workload: str, kernels, per: int):
    """HBM bytes of one table pass (sum over its kernels, one launch each) from the
    committed rocprofv3 PMC summary (profiles/pmc_<workload>.json, made by
    tools/summarize_prof.py from separate FETCH_SIZE and WRITE_SIZE passes of this
    same command), or None when absent or taken at a different shard size."""
    p = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        if d.get("sources_per_launch") != per:
            return None
        return sum(d["kernels"][k]["hbm_bytes_per_launch"] for k in kernels)
    except Exception:
        return None


if __name__ == "__main__":
    main()
