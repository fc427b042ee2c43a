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


def test_env_seeds_are_job_wide():
    """Rank r's env e is job env env0(r) + e and draws from seed + env0(r) + e: the
    seeds of all ranks are disjoint and together equal those of one unsharded batch
    (the reference's one RandomState(seed) per loaded env, manipulation/__init__.py:56-86)."""
    seed, world, n = 12345, 8, 4096
    ids = [distributed.env_seeds(seed, world * n, r, world) for r in range(world)]
    all_ids = np.concatenate([i for i, _ in ids])
    all_seeds = np.concatenate([s for _, s in ids])
    np.testing.assert_array_equal(all_ids, np.arange(world * n))
    np.testing.assert_array_equal(all_seeds, seed + np.arange(world * n))
    assert len(np.unique(all_seeds)) == world * n
    np.testing.assert_array_equal(ids[3][1], seed + 3 * n + np.arange(n))


def _reorient_first_draws(seed, ids):
    """The reference's first-episode reset draws of reorient env `seed + i` for every
    job env i (goal from numpy's global stream, then PropPlacer's position and
    quaternion from the env's RandomState; reorient.py:143-151,182-188,
    prop_orientation.py:34-38), as [len(ids), 4 + 3 + 4] float64."""
    lo, hi = np.array([-0.025, -0.155, 0.16]), np.array([0.025, -0.105, 0.16])
    out = []
    for i in ids:
        g, e = np.random.RandomState(seed + int(i)), np.random.RandomState(seed + int(i))
        rows = []
        for rs in (g, None, e):
            if rs is None:
                rows.append(e.uniform(lo, hi))
                continue
            u1, u2, u3 = rs.uniform([0.0] * 3, [1.0, 2 * np.pi, 2 * np.pi])
            rows.append([np.sqrt(1 - u1) * np.sin(u2), np.sqrt(1 - u1) * np.cos(u2), np.sqrt(u1) * np.sin(u3),
                         np.sqrt(u1) * np.cos(u3)])
        out.append(np.concatenate(rows))
    return np.array(out)


def _gloo_worker(rank, world, port, seed, total, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ids, seeds = distributed.env_seeds(seed, total, rank, world)
        rows = np.concatenate([ids[:, None].astype(np.float64), seeds[:, None].astype(np.float64),
                               _reorient_first_draws(seed, ids)], axis=1)
        # the gathered [W * n, width] buffer: rank r's rows in its own slice (the layout
        # dx_allgather_obs produces in place)
        t = torch.from_numpy(rows)
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        q.put((rank, torch.cat(parts).numpy()))
    finally:
        dist.destroy_process_group()


def test_sharded_job_world2_gloo():
    """Two processes, one shard each, gathered over gloo (a test-only transport standing
    in for the RCCL all-gather): every gathered row holds the job env its slice names,
    the per-env seeds are disjoint across ranks, and the rows -- ids, seeds and the
    reference's reset draws for those seeds -- equal a single-process run of the whole
    job."""
    pytest.importorskip("torch")
    import socket

    world, n, seed = 2, 24, 777
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, seed, world * n, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    np.testing.assert_array_equal(got[0], got[1])
    rows = got[0]
    for r in range(world):
        sl = distributed.gathered_rows(r, n)
        np.testing.assert_array_equal(rows[sl, 0], np.arange(r * n, (r + 1) * n))
    assert len(np.unique(rows[:, 1])) == world * n
    whole = _reorient_first_draws(seed, np.arange(world * n))
    np.testing.assert_array_equal(rows[:, 1], seed + np.arange(world * n))
    np.testing.assert_array_equal(rows[:, 2:], whole)


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
    monkeypatch.delenv("TORCHELASTIC_RESTART_COUNT", raising=False)
    monkeypatch.delenv("TORCHELASTIC_RUN_ID", raising=False)
    assert distributed.job_key() == f"29511_{os.getppid()}_0_"
    # an elastic restart of the same job gets a fresh key (no stale id is read)
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "1")
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "abc-123")
    assert distributed.job_key() == f"29511_{os.getppid()}_1_abc123"


def test_single_node_check(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "16")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    with pytest.raises(RuntimeError):
        distributed.check_single_node()
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "16")
    distributed.check_single_node()


def test_rank0_replaces_stale_id(tmp_path):
    key = "stale"
    (tmp_path / f"dx_comm_{key}.id").write_bytes(b"old")
    got = distributed.exchange_id(0, key, lambda: b"new", directory=str(tmp_path))
    assert got == b"new" and (tmp_path / f"dx_comm_{key}.id").read_bytes() == b"new"
