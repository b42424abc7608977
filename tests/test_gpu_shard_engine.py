"""Multi-rank path with the GPU engine: world size 2, one spawned
process per rank under a gloo group, both ranks on cuda:0 (this box has one GPU;
on a node every rank has its own GPU and the exchange runs over RCCL).

Each rank runs exactly what bench.py runs per rank: Engine.partition of the host
set (the same split on every rank, computed without communicating) ->
part_rows -> Engine.compute_device of its part into device tensors -> the
exchange of shard.combine (all-reduce(MIN) of the row minima, all-gather of the
row shards, rows back in caller order). Rank 0 then computes the whole table on
one engine and asserts that the gathered table and the global minimum equal it
bit for bit. The ranks' kernels are serialised with barriers so each launch has
the GPU to itself, as it has on a node, and the default (wave-model) layout is
the one exercised. Reference: rows are independent in the reference
(_topology_computeSourcePaths, shd-topology.c:775-939, one source at a time).

The complete branch (BASELINE config 3: PlanetLab, all-pairs, sharded) takes the
same path: Engine.partition falls back to balanced blocks on a complete topology
(no landmark embedding), each rank's rows run the direct-edge kernel
(_topology_lookupPath, shd-topology.c:941-979), and the gathered 303 x 303 table
must equal the golden table computed independently from the reference's own
resource/topology.plab.graphml.xml.xz (tests/golden/make_golden.py), at world
sizes 2, 4 and 8 (8 gloo ranks sharing the one GPU of the test box).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q, case, path):
    import torch
    import torch.distributed as dist

    from shadow_amd.routes import Engine, Graph
    from shadow_amd.shard import combine, part_rows

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        if case == "plab":  # complete topology: every vertex a host, direct-edge branch
            g = Graph.load_graphml(path)
            hosts = np.arange(g.V, dtype=np.int32)
        else:
            g = Graph.generate("chunglu", 40_000, 3, 41)
            hosts = np.sort(np.random.default_rng(6).choice(g.V, 6000, replace=False)).astype(np.int32)
        S = T = len(hosts)
        eng = Engine(g, device=0)
        part = eng.partition(hosts, world)
        rows, n_real = part_rows(hosts, part, world, rank)
        lat = torch.empty((len(rows), T), dtype=torch.float64, device=dev)
        rel = torch.empty_like(lat)
        rmin = torch.empty((len(rows),), dtype=torch.float64, device=dev)
        layout = None
        for r in range(world):  # one rank's kernels on the GPU at a time
            if r == rank:
                eng.compute_device(rows, hosts, lat.data_ptr(), rel.data_ptr(), rmin.data_ptr(), None,
                                   stream=torch.cuda.current_stream(dev).cuda_stream)
                torch.cuda.synchronize(dev)
                layout = eng.last_layout()
            dist.barrier()
        # gloo exchanges host tensors (RCCL takes the device tensors directly)
        gmin, lat_all, rel_all = combine(lat.cpu(), rel.cpu(), rmin.cpu(), n_real, S, part=part)
        if rank == 0:
            if case == "plab":
                z = np.load(os.path.join(os.path.dirname(__file__), "golden", "direct_plab.npz"))
                ref_lat, ref_rel = z["lat"], z["rel"]
            else:
                full = Engine(g, device=0).compute(hosts, hosts)
                ref_lat, ref_rel = full.lat, full.rel
            ok_lat = np.array_equal(lat_all.numpy().view(np.uint64), ref_lat.view(np.uint64))
            ok_rel = np.array_equal(rel_all.numpy().view(np.uint64), ref_rel.view(np.uint64))
            ok_min = float(gmin.item()) == float(ref_lat.min())
            q.put((ok_lat, ok_rel, ok_min, float(gmin.item()), layout, np.bincount(part, minlength=world).tolist()))
    finally:
        dist.destroy_process_group()


def _run(world, case, path=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, case, path)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        ok_lat, ok_rel, ok_min, gmin, layout, sizes = q.get(timeout=300)
    finally:
        for p in ps:
            p.join(timeout=120)
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    return ok_lat, ok_rel, ok_min, gmin, layout, sizes


@pytest.mark.timeout(600)
def test_two_rank_engine_shards_equal_one_engine():
    ok_lat, ok_rel, ok_min, gmin, layout, sizes = _run(2, "chunglu")
    assert sizes == [3000, 3000]
    assert ok_lat and ok_rel and ok_min, (ok_lat, ok_rel, ok_min, gmin, layout)
    assert layout["cluster_fallback"] == 0, layout


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_complete_branch_shards_equal_golden_plab(world, topo_paths):
    """BASELINE config 3 ("sharded across 2/4/8 GPUs"): the PlanetLab all-pairs
    table sharded over `world` ranks (blocks of 152/151, 76/76/76/75 or 38 x 7 +
    37 rows) gathers to the golden table bit for bit."""
    ok_lat, ok_rel, ok_min, gmin, layout, sizes = _run(world, "plab", str(topo_paths["plab"]))
    assert sizes == [303 // world + (1 if r < 303 % world else 0) for r in range(world)]
    assert ok_lat and ok_rel and ok_min, (ok_lat, ok_rel, ok_min, gmin)
