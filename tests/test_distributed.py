"""N>1 path on CPU: env sharding, rank seeds, and the packed-output all-gather over
gloo with world_size 2 (the same collator bench.py drives over RCCL)."""

import os
import socket

import numpy as np
import pytest

from dexterity_amd import distributed


def test_env_shard_partitions():
    for total in (1, 7, 4096, 32768, 32769):
        for world in (1, 2, 3, 8):
            if total < world:
                continue
            spans = [distributed.env_shard(total, r, world) for r in range(world)]
            assert spans[0][0] == 0
            for (a0, an), (b0, _) in zip(spans, spans[1:]):
                assert a0 + an == b0
            assert sum(n for _, n in spans) == total
            assert max(n for _, n in spans) - min(n for _, n in spans) <= 1
    assert distributed.env_shard(32768, 3, 8) == (12288, 4096)
    with pytest.raises(ValueError):
        distributed.env_shard(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, width, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        col = distributed.OutputCollator(n, width, device="cpu")
        for step in range(3):
            # rows of rank r at step s: value = 1000*r + 10*s + column, row index in last col
            rows = torch.arange(width, dtype=torch.float32).repeat(n, 1) + 1000 * rank + 10 * step
            rows[:, -1] = torch.arange(n, dtype=torch.float32)
            col.shard.copy_(rows)
            g = col.gather().clone()
            if rank == 0:
                q.put(("gather", step, g.numpy()))
        t = distributed.max_over_ranks(0.5 + rank, "cpu")
        if rank == 0:
            q.put(("max", 0, t))
    finally:
        dist.destroy_process_group()


def test_collator_gloo_world2():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, n, width = 2, 5, 7
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, width, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(4)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    gathers = {s: g for kind, s, g in got if kind == "gather"}
    for step, g in gathers.items():
        assert g.shape == (world * n, width)
        for r in range(world):
            blk = g[r * n:(r + 1) * n]
            np.testing.assert_array_equal(blk[:, 0], 1000 * r + 10 * step)
            np.testing.assert_array_equal(blk[:, -1], np.arange(n))
    assert [v for kind, _, v in got if kind == "max"] == [1.5]
