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


class _DeviceBytes:
    """A raw device allocation seen through __cuda_array_interface__ (torch.as_tensor aliases it)."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "strides": None, "version": 3}


def arena_tensor(engine, device):
    """The engine's weight arena as a uint8 tensor that ALIASES it (no copy): a collective on
    this tensor writes straight into the engine.  `device` is the engine's CUDA device
    (``"cpu"`` only for host-memory stand-ins in CPU tests)."""
    import ctypes

    import torch
    ptr, nbytes = engine.weights_arena()
    dev = torch.device(device)
    if dev.type == "cpu":
        return torch.frombuffer((ctypes.c_uint8 * nbytes).from_address(ptr), dtype=torch.uint8)
    if dev.type != "cuda":
        raise ValueError(f"arena_tensor: the arena lives on a GPU, got device {device}")
    t = torch.as_tensor(_DeviceBytes(ptr, nbytes), device=dev)
    if t.data_ptr() != ptr or t.numel() != nbytes:
        raise RuntimeError("arena_tensor: torch did not alias the weight arena")
    return t


def broadcast_weights(engine, device, group=None, src: int = 0) -> dict:
    """Replicate `src`'s weight arena into every rank's engine with one broadcast, straight
    into the arenas (no staging buffer, no device copies).

    Every rank must have loaded the same model spec and dtype; ranks other than `src` created
    their engine with ``WhisperModelParams(external_weights=True)`` and are committed
    (spt_weights_commit) after the broadcast.  On RCCL (backend "nccl") the arena tensors are
    the collective's buffers; gloo (a one-GPU rehearsal of N ranks) moves the bytes through a
    host copy.  Returns the size and the wall time of the broadcast on this rank.
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
    arena = arena_tensor(engine, device)
    via_host = arena.is_cuda and dist.get_backend(group) == "gloo"
    buf = (arena.cpu() if rank == src else torch.empty(nbytes, dtype=torch.uint8)) if via_host else arena
    if arena.is_cuda:
        torch.cuda.synchronize(arena.device)
    t0 = time.perf_counter()
    dist.broadcast(buf, src=src, group=group)
    if arena.is_cuda:
        torch.cuda.synchronize(arena.device)
    ms = (time.perf_counter() - t0) * 1e3
    if rank != src:
        if via_host:
            arena.copy_(buf)
        engine.commit_weights()
    del buf, arena
    return {"bytes": nbytes, "ms": ms, "path": "host (gloo)" if via_host else "in place"}
