"""Multi-rank path on CPU: world_size 2 (and 3) gloo process groups running the
same sharding + exchange code bench.py uses over RCCL (shadow_amd/shard.py).

Each rank computes its source shard with the CPU oracle (test infrastructure
standing in for the GPU engine here), then all-reduce(MIN) + all-gather; the
gathered table and the global minimum must equal the single-rank oracle table
bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import py_oracle as po
from shadow_amd.shard import combine, shard_rows


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _graph():
    rng = np.random.default_rng(5)
    V = 400
    # random spanning tree + extra edges, continuous weights (unique paths)
    ef = [rng.integers(0, v) for v in range(1, V)]
    et = list(range(1, V))
    for _ in range(600):
        a, b = rng.integers(0, V, 2)
        if a != b:
            ef.append(a)
            et.append(b)
    ef = np.array(ef + list(range(V)), np.int32)
    et = np.array(et + list(range(V)), np.int32)
    lat = rng.uniform(1, 100, len(ef))
    loss = rng.uniform(0, 0.01, len(ef))
    vl = rng.uniform(0, 0.02, V)
    return V, ef, et, lat, loss, vl


def _worker(rank, world, port, S, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        V, ef, et, lat, loss, vl = _graph()
        og = po.OracleGraph(V, ef, et, lat, loss, vl)
        hosts = np.arange(0, V, max(1, V // S), dtype=np.int32)[:S]
        rows, n_real, lo = shard_rows(hosts, world, rank)
        L, R, _, rmin = og.routes(rows, hosts, po.MODE_CANONICAL)
        gmin, lat_all, rel_all = combine(torch.from_numpy(L), torch.from_numpy(R), torch.from_numpy(rmin), n_real,
                                         len(hosts))
        if rank == 0:
            q.put((float(gmin.item()), lat_all.numpy().copy(), rel_all.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,S", [(2, 40), (2, 41), (3, 20)])
def test_sharded_table_equals_single_rank(world, S):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, S, q)) for r in range(world)]
    for p in procs:
        p.start()
    gmin, lat_all, rel_all = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    V, ef, et, lat, loss, vl = _graph()
    og = po.OracleGraph(V, ef, et, lat, loss, vl)
    hosts = np.arange(0, V, max(1, V // S), dtype=np.int32)[:S]
    L, R, _, rmin = og.routes(hosts, hosts, po.MODE_CANONICAL)
    assert lat_all.shape == (len(hosts), len(hosts))
    assert np.array_equal(lat_all.view(np.uint64), L.view(np.uint64))
    assert np.array_equal(rel_all.view(np.uint64), R.view(np.uint64))
    assert gmin == rmin.min()


def test_shard_rows_padding():
    src = np.arange(5, dtype=np.int32)
    got = [shard_rows(src, 4, r) for r in range(4)]
    assert [g[1] for g in got] == [2, 2, 1, 0]
    assert all(len(g[0]) == 2 for g in got)
    cat = np.concatenate([g[0] for g in got])
    assert np.array_equal(cat[:5], src)
    with pytest.raises(ValueError):
        shard_rows(src, 2, 2)
