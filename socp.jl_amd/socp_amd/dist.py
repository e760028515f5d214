"""Multi-GPU sharding: independent problems, contiguous global
index ranges per rank, one process per GPU, and a single collective — the
all-gather of per-problem (status, iters) — over RCCL (backend "nccl") on
MI355X or gloo on the CPU."""
from __future__ import annotations


def shard_range(total: int, rank: int, world: int):
    """Contiguous block [lo, hi) of the global problem index for this rank."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def gather_outcomes(status, iters, group=None):
    """All-gather (status, iters) of every rank's shard; returns int32 [world, B, 2].
    Equal shard sizes (weak scaling) are required by all_gather_into_tensor."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    local = torch.stack([status.to(torch.int32), iters.to(torch.int32)], dim=1).contiguous()
    out = torch.empty((world,) + tuple(local.shape), dtype=torch.int32, device=local.device)
    dist.all_gather_into_tensor(out.view(-1, 2), local, group=group)
    return out
