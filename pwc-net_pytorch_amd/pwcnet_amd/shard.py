"""Data-parallel sharding of the hot path over the GPUs of one node (one process per GPU).

The path shards over independent image pairs: rank r of N takes a contiguous
slice of the global batch and runs the whole warp -> correlation pyramid on it with no
cross-GPU traffic.  The only collectives are outside the data path:

* ``broadcast_module`` -- one RCCL broadcast of a model's parameters from rank 0 over xGMI
  (the Net harness's 20.5 MB of conv weights; the hot-path layers have no parameters),
* ``gather_to`` -- optional gather of per-rank outputs (e.g. final flows) to one rank,
* ``max_over_ranks`` -- the benchmark's barrier-bounded timing (MAX of per-rank elapsed),
* ``all_ranks`` -- every rank's value of a scalar (the benchmark's per-rank timings).

Everything here is backend-agnostic torch.distributed: "nccl" (= RCCL on ROCm) on GPUs,
"gloo" for the CPU tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_bounds(total: int, world: int, rank: int):
    """Contiguous [start, stop) of `total` items for `rank`; the first total % world ranks
    take one extra item.  Every item is owned by exactly one rank."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard(x: torch.Tensor, world: int, rank: int, dim: int = 0) -> torch.Tensor:
    lo, hi = shard_bounds(x.shape[dim], world, rank)
    return x.narrow(dim, lo, hi - lo)


def broadcast_module(module: torch.nn.Module, src: int = 0) -> None:
    """Make every rank's parameters and buffers equal to rank `src`'s (one broadcast each)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src)


def gather_to(x: torch.Tensor, dst: int = 0, dim: int = 0):
    """Concatenate every rank's `x` (shards of possibly different sizes along `dim`) on rank
    `dst`; other ranks get None."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return x
    world = dist.get_world_size()
    n = torch.tensor([x.shape[dim]], device=x.device, dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes)
    if x.shape[dim] < m:  # pad to a common shape for all_gather
        pad = list(x.shape)
        pad[dim] = m - x.shape[dim]
        x = torch.cat([x, x.new_zeros(pad)], dim)
    parts = [torch.empty_like(x) for _ in range(world)]
    dist.all_gather(parts, x.contiguous())
    if dist.get_rank() != dst:
        return None
    return torch.cat([p.narrow(dim, 0, s) for p, s in zip(parts, sizes)], dim)


def max_over_ranks(value: float, device=None) -> float:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_ranks(value: float, device=None) -> list:
    """[value of rank 0, value of rank 1, ...] on every rank (all_gather of one float64)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [value]
    t = torch.tensor([value], dtype=torch.float64, device=device)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [float(p.item()) for p in parts]
