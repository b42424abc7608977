"""RCCL smoke test on MI355X hardware: it shows that RCCL initialises
on the engine's device buffers and runs the exchange's two collectives there; at
world size 1 they are identity copies, so this is NOT coverage of the multi-rank
exchange (the gloo tests, tests/test_shard_gloo.py and test_gpu_shard_engine.py,
cover the N > 1 arithmetic).

bench.py and shadow_amd.shard exchange a pass's results with torch.distributed
"nccl" (= RCCL on ROCm): all-reduce(MIN) of a 1-element f64 device tensor (the
scheduler window's global minimum, shd-topology.c:602-613 / shd-master.c:133-144)
and all_gather_into_tensor of the [rows, T] f64 latency / reliability shards.
The gloo tests cover the N > 1 arithmetic on CPU; this box has one GPU and RCCL
refuses two ranks on one device, so here one rank initialises an RCCL
communicator and runs exactly those two collectives on the engine's device
outputs. At world size 1 they must return their inputs bit for bit.
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


def _worker(port, q):
    import torch
    import torch.distributed as dist

    from shadow_amd.routes import Engine, Graph
    from shadow_amd.shard import local_min

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        g = Graph.generate("chunglu", 3000, 3, 5)
        hosts = np.sort(np.random.default_rng(2).choice(g.V, 96, replace=False)).astype(np.int32)
        S = T = len(hosts)
        lat = torch.empty((S, T), dtype=torch.float64, device=dev)
        rel = torch.empty_like(lat)
        rmin = torch.empty((S,), dtype=torch.float64, device=dev)
        eng = Engine(g, device=0)
        eng.compute_device(hosts, hosts, lat.data_ptr(), rel.data_ptr(), rmin.data_ptr(), None,
                           stream=torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        gmin = local_min(rmin, S)
        before = gmin.clone()
        dist.all_reduce(gmin, op=dist.ReduceOp.MIN)
        lat_all = torch.empty((S, T), dtype=torch.float64, device=dev)
        rel_all = torch.empty_like(lat_all)
        dist.all_gather_into_tensor(lat_all, lat.contiguous())
        dist.all_gather_into_tensor(rel_all, rel.contiguous())
        torch.cuda.synchronize(dev)
        ok = (torch.equal(gmin, before) and torch.equal(lat_all.view(torch.int64), lat.view(torch.int64))
              and torch.equal(rel_all.view(torch.int64), rel.view(torch.int64)))
        q.put((ok, dist.get_backend(), float(gmin.item()), float(lat.min().item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_rccl_exchange_collectives_on_device_outputs():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    try:
        ok, backend, gmin, lat_min = q.get(timeout=240)
    finally:
        p.join(timeout=60)
    assert p.exitcode == 0, p.exitcode
    assert backend == "nccl"
    assert ok
    assert gmin == lat_min  # every host is a target: the row minima's minimum is the table's minimum
