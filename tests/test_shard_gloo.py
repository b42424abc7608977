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
from shadow_amd.shard import combine, gathered_index, part_rows, shard_rows


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


def _balanced_part(S, world, seed):
    """A balanced partition in scrambled order (what Engine.partition returns:
    part sizes S/world or S/world + 1, larger first)."""
    part = np.repeat(np.arange(world), [S // world + (r < S % world) for r in range(world)])
    return np.random.default_rng(seed).permutation(part).astype(np.int32)


def _worker(rank, world, port, S, q, coherent=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        V, ef, et, lat, loss, vl = _graph()
        og = po.OracleGraph(V, ef, et, lat, loss, vl)
        hosts = np.arange(0, V, max(1, V // S), dtype=np.int32)[:S]
        part = _balanced_part(len(hosts), world, 7) if coherent else None
        if coherent:
            rows, n_real = part_rows(hosts, part, world, rank)
        else:
            rows, n_real, lo = shard_rows(hosts, world, rank)
        L, R, _, rmin = og.routes(rows, hosts, po.MODE_CANONICAL)
        gmin, lat_all, rel_all = combine(torch.from_numpy(L), torch.from_numpy(R), torch.from_numpy(rmin), n_real,
                                         len(hosts), part=part)
        if rank == 0:
            q.put((float(gmin.item()), lat_all.numpy().copy(), rel_all.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,S,coherent", [(2, 40, False), (2, 41, False), (3, 20, False), (2, 41, True),
                                              (3, 22, True)])
def test_sharded_table_equals_single_rank(world, S, coherent):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, S, q, coherent)) for r in range(world)]
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


def test_part_rows_and_gathered_index():
    src = np.arange(100, 111, dtype=np.int32)
    part = _balanced_part(11, 3, 1)
    blocks = [part_rows(src, part, 3, r) for r in range(3)]
    assert [b[1] for b in blocks] == [4, 4, 3] and all(len(b[0]) == 4 for b in blocks)
    gathered = np.concatenate([b[0] for b in blocks])
    assert np.array_equal(gathered[gathered_index(part, 3)], src)
    with pytest.raises(ValueError):
        part_rows(src, np.zeros(11, np.int32), 3, 0)  # unbalanced part
