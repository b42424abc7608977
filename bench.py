#!/usr/bin/env python3
"""Benchmark: all-sources latency+reliability route tables on MI355X.

One "step" = one pass of the hot path over one batch: every source row of this
rank x every attached target (shortest path + ordered latency/reliability
epilogue + row minima: one table pass of k_routes_sssp), then the scheduler
window exchange (RCCL all-reduce(MIN) of the global minimum path latency)
across ranks. Inputs (graph CSR, source/target lists) are resident in HBM
before timing; outputs stay in HBM.

Workload (BASELINE.json configs; synthetic data of the named sizes):
  cfg5 (default) synthetic Chung-Lu power law n=1,000,000, 50,000 attached hosts
                 -> 2.5e9 source-paths per step (the north-star table; fits one GPU)
  cfg4           synthetic Barabasi-Albert n=100,000 m=3, 10,000 hosts (1e8 per step)
  cfg2 / cfg3    bundled full / PlanetLab topology, all vertices (direct edge)

Scaling (default "strong", BASELINE configs 4-5 split ONE host set over the
GPUs): rank r computes part r of Engine.partition(hosts, N) (balanced, spatially
coherent parts, identical on every rank), so the whole job computes the S x T
table once per step at every N. --scaling weak
gives every rank S rows of its own instead (rank r's sources are the r-th block
of a seeded vertex permutation whose first block is the host set). The
all-gather of the row shards (every rank receiving the whole table over xGMI) is
timed separately after the timed steps ("allgather").

Besides the timed steps, rank 0 of an N=1 run reports
  cold         a fresh engine's first table: engine upload, landmark pre-pass,
               source grouping and one pass with no measured bucket order
  first_query  the drop-in path as Shadow drives it: topology_new on the
               GraphML file -> topology_attach of every host (exact-IP hint)
               -> the first topology_getLatency (engine + table + host copy)
  cpu_baseline the oracle (igraph-style Dijkstra + epilogue) on the host cores
  side_configs cfg4 and the bundled complete topologies (cfg2 / cfg3)

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg5]
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

from shadow_amd.routes import SHDR_TIMING, Engine, Graph, lib_kernel_sha, src_kernel_sha  # noqa: E402
from shadow_amd.shard import allgather_rows, allreduce_min, local_min, part_rows  # noqa: E402

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


def rank_sources(eng, hosts, pool, world, rank, scaling):
    """-> (rows padded, n_real): this rank's source rows. Strong scaling splits the
    host set by Engine.partition (balanced, spatially coherent parts, identical on
    every rank), so each rank's buckets group as tightly as one GPU's would."""
    if scaling == "strong":
        if world == 1:
            return hosts, len(hosts)
        return part_rows(hosts, eng.partition(hosts, world), world, rank)
    S = len(hosts)
    if rank == 0:
        return hosts, S
    if (rank + 1) * S <= len(pool):
        return np.sort(pool[rank * S:(rank + 1) * S]), S
    # not enough distinct vertices for a disjoint block: cycle through the pool
    idx = (np.arange(S) + rank * S) % len(pool)
    return np.sort(pool[idx]), S


def cpu_threads() -> int:
    """The host cores this process may use: OMP_NUM_THREADS (set to the box's CPU
    share per GPU on the GPU pool: nproc there counts the whole machine), else the
    affinity mask."""
    try:
        n = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        n = 0
    return max(1, n or len(os.sched_getaffinity(0)))


CPU_SAMPLE_SEED = 1


def cpu_baseline(g: Graph, hosts: np.ndarray, complete: bool, budget_s: float = 30.0) -> dict:
    """Reference-faithful CPU path (oracle restatement of igraph Dijkstra + the
    epilogue, or the direct edge) on ONE core, on a bounded, seeded random sample
    of sources (numpy default_rng(CPU_SAMPLE_SEED) permutation of the hosts, the
    first n of it) x every target; then the same port
    source-parallel over this process's CPU share."""
    from oracle import py_oracle as po  # test infrastructure: the baseline, never the measured path

    og = po.OracleGraph.from_graph(g)
    mode = po.MODE_COMPLETE if complete else po.MODE_IGRAPH
    T = len(hosts)
    sample = hosts[np.random.default_rng(CPU_SAMPLE_SEED).permutation(len(hosts))]
    n = min(2, len(hosts))
    t0 = time.perf_counter()
    og.routes(sample[:n], hosts, mode, threads=1)
    dt = time.perf_counter() - t0
    n2 = int(min(len(hosts), max(n, budget_s / max(dt / n, 1e-9))))
    if n2 > n:
        t0 = time.perf_counter()
        og.routes(sample[:n2], hosts, mode, threads=1)
        dt = time.perf_counter() - t0
        n = n2
    out = {"value": n * T / dt, "unit": "source-paths/s", "cores": 1, "kind": "port",
           "sample": f"{n} of {len(hosts)} sources (seeded random sample: default_rng({CPU_SAMPLE_SEED}) permutation "
                     f"of the hosts) x {T} targets, {dt:.1f} s on 1 core "
                     f"({'direct edge' if complete else 'binary-heap Dijkstra + ordered epilogue'}); "
                     "extrapolation: sources are independent. 1 core is reference-faithful: the reference "
                     "serialises Dijkstra under graphLock (shd-topology.c:859-893). The sample is sized to "
                     f"~{budget_s:.0f} s of CPU work (the bench contract bounds the CPU leg to 10-30 s so the "
                     "default run ends in minutes); the all_cores leg runs BASELINE.md's 256 sources",
           "seed": CPU_SAMPLE_SEED}
    cores = cpu_threads()
    if cores > 1 and not complete:
        # at least the 256 seeded sources BASELINE.md plans (about 0.5 x the 1-core budget of wall time)
        m = int(min(len(hosts), max(256, cores, n * cores * 0.5)))
        t0 = time.perf_counter()
        og.routes(sample[:m], hosts, mode, threads=cores)
        dt2 = time.perf_counter() - t0
        nproc = os.cpu_count()
        out["all_cores"] = {"value": m * T / dt2, "cores": cores, "nproc": nproc,
                            "label": f"{cores} of {nproc} host threads (per-GPU share)",
                            "sample": f"the first {m} sources of the same seeded sample x {T} targets, {dt2:.1f} s on "
                                      f"{cores} threads (cores = OMP_NUM_THREADS / affinity: this process's CPU "
                                      "share, 16 per GPU on the GPU pool)"}
    return out


def kernel_sha() -> str:
    """sha of the library sources in the tree (routes.hip + the host code around it)"""
    return src_kernel_sha()


def check_lib_sha() -> str:
    """The loaded library's compiled-in source sha; a library built from other
    sources than the tree's would put this tree's sha on another build's numbers,
    so the bench refuses to run then."""
    lib = lib_kernel_sha()
    if lib != kernel_sha():
        raise SystemExit(f"bench: libshdtopology.so was built from sources {lib}, the tree holds {kernel_sha()}: "
                         "rebuild (make -C shadow_amd)")
    return lib


def load_pmc_traffic(workload: str, kernels, per: int):
    """HBM bytes of one table pass (sum over its kernels, one launch each) from the
    committed rocprofv3 PMC summary (profiles/pmc_<workload>.json, made by
    tools/summarize_prof.py from separate FETCH_SIZE and WRITE_SIZE passes of this
    same command), or None when absent, taken at a different shard size, or taken
    with a different routes.hip (sha recorded by tools/profile.sh)."""
    p = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        if d.get("sources_per_launch") != per or d.get("kernel_sha") != kernel_sha():
            return None
        return sum(d["kernels"][k]["hbm_bytes_per_launch"] for k in kernels)
    except Exception:
        return None


def eng_arcs(g: Graph) -> int:
    ef, et, _, _, _ = g.export()
    loops = int((ef == et).sum())
    return (len(ef) - loops) * (1 if g.directed else 2)


def algorithmic_bytes(complete: bool, rows: int, T: int, V: int, A: int) -> float:
    """SSSP 12 B/arc + 20 B/vertex per source row + 16 B/pair;
    direct edge 32 B/pair."""
    if complete:
        return 32.0 * rows * T
    return rows * (12.0 * A + 20.0 * V) + 16.0 * rows * T


def first_query(g: Graph, hosts: np.ndarray) -> dict:
    """topology_new (GraphML) -> attach every host -> first getLatency, through the
    drop-in (include/shd_topology.h) exactly as Shadow calls it at start-up
    (shd-master.c:209, shd-host.c:277, shd-worker.c:246). The first query builds
    the whole table (engine upload, landmark pre-pass, pass, D2H)."""
    from shadow_amd import topology as top

    fd, path = tempfile.mkstemp(suffix=".graphml.xml", dir="/tmp")
    os.close(fd)
    t0 = time.perf_counter()
    g.save_graphml(path)
    write_s = time.perf_counter() - t0
    size = os.path.getsize(path)
    ips = [g.vertex_str("ip", int(v)) for v in hosts]
    addrs = [top.Address(f"11.{(i >> 16) & 255}.{(i >> 8) & 255}.{i & 255}", f"host{i}") for i in range(len(hosts))]
    rnd = top.Random(1)
    t0 = time.perf_counter()
    t = top.Topology.new(path)
    t1 = time.perf_counter()
    os.unlink(path)  # Shadow unlinks the temp topology file right after topology_new (shd-master.c:210)
    if t is None:
        return {"error": "topology_new failed"}
    for a, ip in zip(addrs, ips):
        t.attach(a, rnd, ip_hint=ip)
    t2 = time.perf_counter()
    lat = t.get_latency(addrs[0], addrs[-1])
    t3 = time.perf_counter()
    lat2 = t.get_latency(addrs[-1], addrs[0])
    t4 = time.perf_counter()
    placed = all(t.vertex_of(addrs[i]) == int(hosts[i]) for i in range(0, len(hosts), max(1, len(hosts) // 100)))
    phases = t.last_compute_times()
    nblk, rows_per_block, _ = t.table_blocks()
    t.free()
    return {"total_ms": (t3 - t0) * 1e3, "topology_new_ms": (t1 - t0) * 1e3, "attach_ms": (t2 - t1) * 1e3,
            "first_get_latency_ms": (t3 - t2) * 1e3, "next_get_latency_us": (t4 - t3) * 1e6,
            "hosts": len(hosts), "graphml_bytes": size, "graphml_write_s_untimed": write_s,
            "phases": {"engine_create_ms": phases["engine_create_ms"], "landmarks_ms": phases["landmarks_ms"],
                       "grouping_ms": phases["grouping_ms"], "launch_ms": phases["launch_ms"],
                       "pass_ms": phases["pass_ms"], "d2h_ms": phases["d2h_ms"],
                       "table_ms": phases["block_ms"],
                       "note": "engine_create runs in a background thread started by topology_new, so it "
                               "overlaps the attach calls; first getLatency = the part of engine_create still "
                               "running + table_ms; table_ms = landmarks (the pre-pass enqueued by engine_create, "
                               "collected here) + grouping + launch (uploads, arena, kernel enqueue) + pass "
                               "(kernels; the host pre-faults the table meanwhile) + d2h (exposed copy)"},
            "table_blocks": nblk, "rows_per_block": rows_per_block,
            "hosts_on_bench_vertices": placed, "latency_ms_first_pair": lat, "latency_ms_reverse": lat2,
            "note": "first_get_latency = what remains of the engine start-up (background since topology_new) + "
                    "one table pass + D2H of the S x T latency/reliability table into the drop-in's host table"}


def run(name, *, steps, warmup, world, rank, local, dev, scaling, backend, gather, cold):
    g, hosts, pool, desc = make_workload(name)
    info = g.check()
    complete = bool(info.is_complete)
    T = len(hosts)
    S_total = T * world if scaling == "weak" else T
    stream = torch.cuda.current_stream(dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    eng = Engine(g, device=local)
    torch.cuda.synchronize(dev)
    create_ms = (time.perf_counter() - t0) * 1e3
    mine, n_real = rank_sources(eng, hosts, pool, world, rank, scaling)
    per = len(mine)
    lat = torch.empty((per, T), dtype=torch.float64, device=dev)
    rel = torch.empty((per, T), dtype=torch.float64, device=dev)
    rmin = torch.empty((per,), dtype=torch.float64, device=dev)
    gmin = torch.empty((1,), dtype=torch.float64, device=dev)
    kernel_ms = []  # per timed step: {kernel name: ms} (HIP events on the launch stream)

    def step(record: bool):
        eng.compute_device(mine, hosts, lat.data_ptr(), rel.data_ptr(), rmin.data_ptr(), None, flags=SHDR_TIMING,
                           stream=stream.cuda_stream)
        if record:
            kernel_ms.append(eng.timing())
        gmin.copy_(allreduce_min(local_min(rmin, n_real)))

    # cold: this engine's first table (landmark pre-pass + grouping + one pass, no measured order)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    step(False)
    torch.cuda.synchronize(dev)
    cold_ms = (time.perf_counter() - t0) * 1e3
    cold_t = eng.timing()
    cold_pass = cold_t.get("routes_pass")
    for _ in range(warmup):
        step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    gather_rec = None
    if world > 1 and gather:
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
        gather_rec = {"allgather_ms": float(tgm.item()) * 1e3, "table_bytes_per_rank": gbytes,
                      "value_incl_gather": S_total * T / (elapsed / steps + float(tgm.item()))}
        del lat_all, rel_all

    V = info.vertex_count
    A = int(eng_arcs(g))
    names = sorted({k for d in kernel_ms for k in d if k != "routes_pass" and not k.startswith("host_")})
    per_kernel = {k: float(np.mean([d.get(k, 0.0) for d in kernel_ms])) for k in names}
    # One table pass = the main launch (+ a narrower tail launch for the partial last wave of
    # buckets, concurrent on a second stream, routes.hip): bytes and time over the pass, fork to join.
    passes = [d["routes_pass"] for d in kernel_ms if "routes_pass" in d]
    k_ms = float(np.mean(passes)) if passes else (sum(per_kernel.values()) if per_kernel else float("nan"))
    bytes_per_launch = algorithmic_bytes(complete, per, T, V, A)
    achieved = bytes_per_launch / (k_ms * 1e-3) / 1e9
    res = {
        "metric": "source-paths/sec (all-sources latency+reliability)",
        "value": S_total * T * steps / elapsed,
        "unit": "source-paths/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": elapsed / steps * 1e3,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic" if name in ("cfg4", "cfg5") else "reference bundled topology",
        "config": dict(desc, V=V, arcs=A, sources=S_total, targets=T, sources_per_rank=per,
                       parallelism=f"source-shard x{world}" + (
                           f" + {'RCCL' if backend == 'nccl' else backend} all-reduce(MIN)" if world > 1 else ""),
                       branch="direct-edge" if complete else "shortest-path"),
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": load_pmc_traffic(name, names, per),
                     "kernel": " + ".join(names), "kernel_ms": k_ms, "kernel_ms_each": per_kernel,
                     "kernel_ms_note": ("kernel_ms = one table pass = one launch (HIP events on its stream)"
                                        if len(names) == 1 else
                                        "kernel_ms = one table pass, fork to join; the tail launch overlaps the main "
                                        "launch (its time is counted from the fork)"),
                     "algorithmic_bytes_per_launch": bytes_per_launch,
                     "algorithmic_bytes_model": "direct: 32 B/pair" if complete else
                     "per source row 12 B/arc (col + weight) + 20 B/vertex (rowptr + dist + pred) + 16 B/pair",
                     "kernel_sha": kernel_sha(), "lib_sha": check_lib_sha()},
        "global_min_latency_ms": float(gmin.item()),
    }
    if not complete:  # bucket layout this rank's engine chose (schedule only: shdr_engine_last_layout)
        res["layout"] = eng.last_layout()
    if cold:
        res["cold"] = {"engine_create_ms": create_ms, "first_table_ms": cold_ms, "first_pass_kernel_ms": cold_pass,
                       "phases": {k[5:] + "_ms": v for k, v in cold_t.items() if k.startswith("host_")},
                       "value": S_total * T / (cold_ms * 1e-3),
                       "note": "a fresh engine's first table: landmark pre-pass + source grouping + one pass "
                               "(no measured bucket order); the timed steps reuse the cached grouping and "
                               "issue buckets in the same spread order, or, for a main launch of at most 4 "
                               "waves of buckets (strong-scaling shards), longest-measured-first from the "
                               "previous pass (SHDR_PROFILE_ORDER: 1 always, 0 never)"}
    if gather_rec:
        res["allgather"] = gather_rec
    del eng, lat, rel, rmin
    torch.cuda.empty_cache()
    return res, g, hosts, complete


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default=os.environ.get("SHDR_BENCH_WORKLOAD", "cfg5"))
    ap.add_argument("--scaling", choices=["weak", "strong"], default="strong")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-first-query", action="store_true")
    ap.add_argument("--no-gather", action="store_true", help="skip the (separately timed) all-gather")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL; gloo only "
                    "to rehearse the multi-rank flow with every rank on one GPU, --same-device)")
    ap.add_argument("--same-device", action="store_true", help="every rank uses cuda:0 (rehearsal)")
    ap.add_argument("--no-side-configs", action="store_true", help="skip the cfg4 / bundled-topology side lines")
    args = ap.parse_args()

    check_lib_sha()
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

    result, g, hosts, complete = run(args.workload, steps=args.steps, warmup=args.warmup, world=world, rank=rank,
                                     local=local, dev=dev, scaling=args.scaling, backend=args.backend,
                                     gather=not args.no_gather, cold=True)
    solo = rank == 0 and world == 1
    if solo and not args.no_first_query and args.workload in ("cfg4", "cfg5"):
        result["first_query"] = first_query(g, hosts)
    if solo and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(g, hosts, complete)
    if solo and not args.no_side_configs:
        side = {}
        for name in ("cfg4", "cfg5", "cfg2", "cfg3"):
            if name == args.workload:
                continue
            if name == "cfg5":
                continue  # the headline; as a side line it would double the run
            r, *_ = run(name, steps=5 if name == "cfg4" else 50, warmup=1, world=1, rank=0, local=local, dev=dev,
                        scaling="strong", backend=args.backend, gather=False, cold=False)
            side[name] = {k: r[k] for k in ("value", "unit", "ms_per_step", "steps")}
            side[name]["workload"] = r["config"]["workload"]
            side[name]["roofline_frac"] = r["roofline"]["frac"]
            side[name]["kernel_ms"] = r["roofline"]["kernel_ms"]
        result["side_configs"] = side
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
