"""Source sharding of the all-sources route table over ranks (one process per GPU).

The reference computes one source row at a time on one core
(_topology_computeSourcePaths, /root/reference/src/main/routing/shd-topology.c:775-939,
serialised under graphLock :859-893).  Rows are independent, so here the S
attached sources are split into W contiguous shards of ceil(S/W) rows, one per
rank; every rank holds a full replica of the CSR graph and computes its shard
on its own GPU.  The path has exactly two exchange steps, both after compute:

  * the scheduler window input (the minimum over every stored path latency,
    _topology_storePathInCache :602-613 -> master_updateMinTimeJump
    shd-master.c:133-144): all-reduce(MIN) of one f64 per rank;
  * the table itself, when every rank needs every row: all-gather of the
    per-rank [ceil(S/W), T] latency and reliability shards.

On ROCm the "nccl" backend is RCCL over xGMI; tests drive the same code with
"gloo" on CPU tensors.  The last shard is padded with copies of its last real
row so every rank contributes an equal-size block; padded rows are excluded from
the minimum and dropped after the gather. For strong scaling the split can instead
follow Engine.partition (balanced, spatially coherent parts: each rank's bucket
grouping stays as tight as the whole list's); part_rows / gathered_index map
those rows back to the caller's order.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def shard_rows(sources: np.ndarray, world: int, rank: int) -> tuple[np.ndarray, int, int]:
    """-> (rows[per] int32 padded, n_real, first row index) for this rank."""
    sources = np.ascontiguousarray(sources, dtype=np.int32)
    S = len(sources)
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    per = max(1, -(-S // world))
    lo = min(rank * per, S)
    rows = sources[lo:lo + per]
    n_real = len(rows)
    if n_real < per:
        fill = sources[-1] if S else 0
        rows = np.concatenate([rows, np.full(per - n_real, fill, np.int32)])
    return rows, n_real, lo


def part_rows(sources: np.ndarray, part: np.ndarray, world: int, rank: int) -> tuple[np.ndarray, int]:
    """-> (rows[per] int32 padded, n_real): the sources of part `rank` of a
    strong-scaling partition (Engine.partition: balanced, spatially coherent, the
    same on every rank), in caller order, padded to per = ceil(S/world) rows with
    copies of their last row so every rank contributes an equal block."""
    sources = np.ascontiguousarray(sources, dtype=np.int32)
    part = np.asarray(part)
    if world < 1 or not 0 <= rank < world or part.shape != sources.shape:
        raise ValueError("bad partition")
    S = len(sources)
    per = max(1, -(-S // world))
    rows = sources[part == rank]
    n_real = len(rows)
    if n_real > per:
        raise ValueError("partition part larger than ceil(S/world)")
    if n_real < per:
        fill = rows[-1] if n_real else (sources[-1] if S else 0)
        rows = np.concatenate([rows, np.full(per - n_real, fill, np.int32)])
    return rows, n_real


def gathered_index(part: np.ndarray, world: int) -> np.ndarray:
    """idx[i] = row of source i (caller order) in the rank-major all-gather of
    part_rows blocks; table_in_caller_order = gathered[idx]."""
    part = np.asarray(part)
    S = len(part)
    per = max(1, -(-S // world))
    idx = np.empty(S, np.int64)
    for r in range(world):
        pos = np.nonzero(part == r)[0]
        idx[pos] = r * per + np.arange(len(pos))
    return idx


def local_min(row_min: torch.Tensor, n_real: int) -> torch.Tensor:
    """Minimum over this rank's real rows as a 1-element tensor (+inf if none)."""
    if n_real <= 0:
        return torch.full((1,), float("inf"), dtype=row_min.dtype, device=row_min.device)
    return row_min[:n_real].min().reshape(1)


def allreduce_min(gmin: torch.Tensor, group=None) -> torch.Tensor:
    """In-place global minimum across ranks (RCCL/gloo all-reduce MIN)."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(gmin, op=dist.ReduceOp.MIN, group=group)
    return gmin


def allgather_rows(shard: torch.Tensor, out: torch.Tensor | None = None, group=None) -> torch.Tensor:
    """Concatenate equal-size [per, T] row shards of every rank into [W*per, T]."""
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return shard if out is None else out.copy_(shard)
    W = dist.get_world_size(group)
    if out is None:
        out = torch.empty((W * shard.shape[0],) + tuple(shard.shape[1:]), dtype=shard.dtype, device=shard.device)
    if dist.get_backend(group) == "gloo":
        # gloo has no single-buffer (or device) all-gather: list all-gather on host copies
        parts = [torch.empty(shard.shape, dtype=shard.dtype) for _ in range(W)]
        dist.all_gather(parts, shard.detach().cpu().contiguous(), group=group)
        out.copy_(torch.cat(parts, dim=0))
    else:
        dist.all_gather_into_tensor(out, shard.contiguous(), group=group)
    return out


def combine(lat: torch.Tensor, rel: torch.Tensor, row_min: torch.Tensor, n_real: int, S: int,
            gather: bool = True, group=None, part: np.ndarray | None = None):
    """Exchange step of one table pass: -> (global min latency, lat[S,T] | None, rel[S,T] | None).
    Rows come from shard_rows (contiguous blocks) or, with `part`, from part_rows;
    the gathered table is returned in the caller's row order either way."""
    gmin = allreduce_min(local_min(row_min, n_real), group)
    if not gather:
        return gmin, None, None
    lat_all = allgather_rows(lat, group=group)
    rel_all = allgather_rows(rel, group=group)
    if part is None:
        return gmin, lat_all[:S], rel_all[:S]
    W = dist.get_world_size(group) if dist.is_initialized() else 1
    idx = torch.as_tensor(gathered_index(part, W), device=lat_all.device)
    return gmin, lat_all.index_select(0, idx), rel_all.index_select(0, idx)
