"""N>1 path on CPU (no GPU, no torch): env sharding, rank seeds, the gathered-buffer
layout, and the communicator-id bootstrap between two processes (the file exchange
every rank of a torch.distributed.run job performs before dx_comm_init).  The RCCL
all-gather itself runs on the GPU (tests/test_gpu_parity.py::test_allgather_world1)."""

import multiprocessing as mp
import os

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


def test_gathered_rows_cover_the_job():
    world, n = 8, 4096
    seen = np.zeros(world * n, dtype=int)
    for r in range(world):
        sl = distributed.gathered_rows(r, n)
        assert sl.start == distributed.env_shard(world * n, r, world)[0]
        seen[sl] += 1
    assert np.all(seen == 1)
    assert distributed.rank_seed(12345, 3) == 12348


def _exchange_worker(rank, key, directory, q):
    def make_id():
        return bytes(range(128))[::-1] if rank == 0 else b"wrong"

    q.put((rank, distributed.exchange_id(rank, key, make_id, timeout=60, directory=directory)))


def test_id_exchange_world2(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    key = f"test_{os.getpid()}"
    # rank 1 starts first: it must wait for rank 0's file, never read a partial one
    procs = [ctx.Process(target=_exchange_worker, args=(r, key, str(tmp_path), q)) for r in (1, 0)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0] == got[1] == bytes(range(128))[::-1]
    distributed.cleanup_id(key, str(tmp_path))
    assert not list(tmp_path.iterdir())


def test_id_exchange_times_out(tmp_path):
    with pytest.raises(TimeoutError):
        distributed.exchange_id(1, "nobody", lambda: b"", timeout=0.2, directory=str(tmp_path))


def test_job_key_is_shared_by_launcher_children(monkeypatch):
    monkeypatch.setenv("MASTER_PORT", "29511")
    assert distributed.job_key() == f"29511_{os.getppid()}"
