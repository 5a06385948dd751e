"""World-size-2 gloo tests (CPU) of the replica-parallel plumbing used by bench.py --gpus N:
utterance shards cover every item exactly once, gathered results keep global order, and
the timing reduction is the max over ranks."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from spittle_amd.dist import shard_range


def test_shard_range_partitions():
    for n in (0, 1, 7, 8, 64, 65):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                b, e = shard_range(n, world, r)
                assert 0 <= b <= e <= n
                seen.extend(range(b, e))
            assert seen == list(range(n))
            sizes = [shard_range(n, world, r)[1] - shard_range(n, world, r)[0] for r in range(world)]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from spittle_amd.dist import max_over_ranks, run_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    items = [f"utt{i}" for i in range(13)]
    calls = []

    def fn(shard):
        calls.append(list(shard))
        return [s.upper() + f"@{rank}" for s in shard]

    out = run_sharded(fn, items)
    t = max_over_ranks(1.0 + rank)
    q.put((rank, out, calls, t))
    dist.barrier()
    dist.destroy_process_group()


def test_run_sharded_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    expected = [f"UTT{i}@{0 if i < 7 else 1}" for i in range(13)]
    for rank, out, calls, t in res:
        assert out == expected                      # same ordered result on every rank
        assert len(calls) == 1                      # each rank ran only its own shard
        b, e = shard_range(13, world, rank)
        assert calls[0] == [f"utt{i}" for i in range(b, e)]
        assert t == 2.0                             # max over ranks


class _HostArenaEngine:
    """Stand-in for WhisperEngine's weight-arena calls on CPU memory (the host logic of
    broadcast_weights; the device path is covered by the -m gpu tests)."""

    def __init__(self, nbytes, fill=None):
        import numpy as np
        self.arena = np.zeros(nbytes, np.uint8) if fill is None else fill.copy()
        self.committed = fill is not None

    def info(self):
        return {"weight_bytes": self.arena.size}

    def weights_arena(self):
        return self.arena.ctypes.data, self.arena.size

    def commit_weights(self):
        self.committed = True


def _bcast_worker(rank, world, port, q, sizes):
    import numpy as np
    import torch.distributed as dist
    from spittle_amd.dist import broadcast_weights
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = sizes[rank]
    src = np.random.default_rng(7).integers(0, 256, n, dtype=np.uint8)
    eng = _HostArenaEngine(n, fill=src if rank == 0 else None)
    try:
        info = broadcast_weights(eng, device="cpu")
        q.put((rank, "ok", bool((eng.arena == src).all()) and eng.committed, info["bytes"]))
    except RuntimeError as e:
        q.put((rank, "err", str(e), 0))
    dist.barrier()
    dist.destroy_process_group()


def _run_bcast(sizes):
    world, port = len(sizes), _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_bcast_worker, args=(r, world, port, q, sizes)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_broadcast_weights_gloo_world2():
    """Rank 0's arena lands byte for byte in rank 1's (external-weights) engine."""
    n = 3 * 1024 * 1024 + 17
    for rank, kind, same, nbytes in _run_bcast([n, n]):
        assert kind == "ok" and same and nbytes == n, (rank, kind, same)


def test_broadcast_weights_size_mismatch_fails_loudly():
    """Engines of different models (arena sizes) refuse the broadcast on every rank."""
    for rank, kind, msg, _ in _run_bcast([4096, 8192]):
        assert kind == "err" and "disagree" in msg, (rank, kind, msg)
