"""One-process-per-GPU replica helpers (images shard with no exchange step).

The only cross-rank traffic is control: a barrier around the timed region and
the max of the per-rank elapsed times (gloo on the host; no RCCL on the data
path). `shard(n, rank, world)` splits a stream of independent images.
"""
from __future__ import annotations

import os


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(n: int, rank: int, world: int) -> range:
    """Contiguous, balanced split of n independent items over `world` replicas."""
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def max_over_ranks(x: float) -> float:
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_gather_obj(obj) -> list:
    """Every rank's `obj` (rank order) over the gloo control group; [obj] without one."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def barrier():
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()
