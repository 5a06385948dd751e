"""Multi-GPU plumbing: utterance sharding for replica-parallel transcription.

Whisper windows are independent, so N GPUs run N independent engines,
one process per GPU (torchrun / torch.distributed, RCCL backend on ROCm). No collective
sits on the data path: a rank transcribes its contiguous shard; results are gathered on
the host only when the caller wants them on one rank, and the benchmark takes the max of
the per-rank wall times.
"""
from __future__ import annotations

from typing import Callable, List, Sequence, Tuple


def shard_range(n_items: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced [begin, end) of `n_items` for `rank` of `world`."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    base, rem = divmod(n_items, world)
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


def run_sharded(fn: Callable[[Sequence], list], items: Sequence, group=None) -> List:
    """Apply `fn` to this rank's shard of `items`; return the full, ordered result list
    on every rank (host-side all_gather of Python objects)."""
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return list(fn(items))
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    b, e = shard_range(len(items), world, rank)
    mine = list(fn(items[b:e])) if e > b else []
    parts: List = [None] * world
    dist.all_gather_object(parts, mine, group=group)
    return [r for p in parts for r in p]


def max_over_ranks(value: float, device=None, group=None) -> float:
    """Max of a per-rank scalar (wall time) over the process group."""
    import torch
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
