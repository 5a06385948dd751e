"""Multi-GPU plumbing: utterance sharding for replica-parallel transcription.

Whisper windows are independent, so N GPUs run N independent engines,
one process per GPU (torchrun / torch.distributed, RCCL backend on ROCm). No collective
sits on the data path: a rank transcribes its contiguous shard; results are gathered on
the host only when the caller wants them on one rank, and the benchmark takes the max of
the per-rank wall times.

The one collective is at load time: rank 0 loads the model (file parse and
device dequantisation, or synthetic generation) and its weight arena is broadcast over RCCL
(xGMI) into the engines of the other ranks, which were created with external weights.
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


def broadcast_weights(engine, device=None, group=None, src: int = 0) -> dict:
    """Replicate `src`'s weight arena into every rank's engine with one broadcast.

    Every rank must have loaded the same model spec and dtype; ranks other than `src` created
    their engine with ``WhisperModelParams(external_weights=True)``.  The arena travels as one
    uint8 tensor (RCCL on GPU tensors; gloo also works, via the host).  Returns the size and
    the wall time of the broadcast on this rank.
    """
    import time

    import torch
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return {"bytes": 0, "ms": 0.0}
    rank = dist.get_rank(group)
    nbytes = int(engine.info()["weight_bytes"])
    sizes = [None] * dist.get_world_size(group)
    dist.all_gather_object(sizes, nbytes, group=group)
    if len(set(sizes)) != 1:
        raise RuntimeError(f"broadcast_weights: ranks disagree on the weight arena size: {sizes}")
    buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
    if rank == src:
        engine.export_weights(buf.data_ptr(), nbytes)
    if buf.is_cuda:
        torch.cuda.synchronize(buf.device)
    t0 = time.perf_counter()
    dist.broadcast(buf, src=src, group=group)
    if buf.is_cuda:
        torch.cuda.synchronize(buf.device)
    ms = (time.perf_counter() - t0) * 1e3
    if rank != src:
        engine.import_weights(buf.data_ptr(), nbytes)
    del buf
    return {"bytes": nbytes, "ms": ms}
