"""Multi-GPU sharding and observation collation, torch-free.

Environments are independent. Rank r of W owns the contiguous env range
`env_shard(B_global, r, W)` on its own GPU and steps it with no data-path collective.
Its dx_env is created with `env_offset` = the range's first env, so every per-env
stream (reset draws, device-sampled actions) is keyed by the job-wide env index.
The only exchange is one all-gather per control step of each rank's packed
`[obs | reward | discount | step_type]` rows. That gather is `dx_allgather_obs` in
libdx, which calls RCCL (librccl) directly over xGMI: about 2 MB per rank at 4096 envs.

Bootstrap: rank 0 creates the RCCL unique id (`dx_comm_unique_id`) and publishes it
in a file named by the job key. Every rank reads it before `dx_comm_init`. A job
launched by `torch.distributed.run` (the bench contract's launcher) gives every rank
the same MASTER_PORT and the same parent process (the launcher's agent), so
`job_key()` is unique per job without any extra rendezvous. The launcher is the only
torch component involved, and nothing here imports torch.
"""

from __future__ import annotations

import ctypes
import os
import tempfile
import time
from typing import Callable, Optional, Tuple

from dexterity_amd import _lib


def env_shard(global_envs: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [env0, env0 + n) of rank `rank`; the first `global_envs % world`
    ranks take one extra env."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, extra = divmod(global_envs, world)
    n = base + (1 if rank < extra else 0)
    env0 = rank * base + min(rank, extra)
    return env0, n


def env_seeds(seed: int, global_envs: int, rank: int, world: int):
    """Global env ids and reset-stream seeds of rank `rank`'s shard.

    The reference loads one environment per process with one RandomState
    (manipulation/__init__.py:56-86); a batch of them here gives env i of the job the
    seed `seed + i` (include/dx.h dx_env_create_shard), whichever rank steps it.  Rank r
    creates its dx_env with env_offset = env0(r), so the seeds of a sharded job are
    disjoint across ranks and equal those of one unsharded batch of all the envs."""
    import numpy as np

    env0, n = env_shard(global_envs, rank, world)
    ids = np.arange(env0, env0 + n, dtype=np.int64)
    return ids, (int(seed) + ids) & 0xFFFFFFFF


def gathered_rows(rank: int, n_per_rank: int) -> slice:
    """Rows of the gathered [W * n, width] buffer that hold rank `rank`'s envs (the
    in-place all-gather of dx_allgather_obs packs each rank into its own slice)."""
    return slice(rank * n_per_rank, (rank + 1) * n_per_rank)


def job_key() -> str:
    """Same string on every rank of one launcher attempt, different across jobs and
    across the elastic restarts of one job (torchrun keeps MASTER_PORT and the agent
    pid over --max-restarts, so the restart count and run id are part of the key: a
    rank of a new attempt never reads an id file a failed attempt left behind)."""
    attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
    run = "".join(ch for ch in os.environ.get("TORCHELASTIC_RUN_ID", "") if ch.isalnum())[:32]
    return f"{os.environ.get('MASTER_PORT', '0')}_{os.getppid()}_{attempt}_{run}"


def check_single_node() -> None:
    """The id file lives in this node's temp directory: every rank must be on one node."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world != local:
        raise RuntimeError(f"WORLD_SIZE {world} != LOCAL_WORLD_SIZE {local}: the communicator bootstrap "
                           "(a node-local id file) supports one node")


def exchange_id(rank: int, key: str, make_id: Callable[[], bytes], timeout: float = 120.0,
                directory: Optional[str] = None) -> bytes:
    """Rank 0 calls make_id() and publishes the bytes; every rank returns them.

    The file is written to a temporary name and renamed, so a reader never sees a
    partial id. Rank 0 removes the file once the id is consumed (on the next call with
    the same key, or at exit of the job through `cleanup_id`)."""
    directory = directory or tempfile.gettempdir()
    path = os.path.join(directory, f"dx_comm_{key}.id")
    if rank == 0:
        try:  # never leave an older id where a reader could take it
            os.remove(path)
        except FileNotFoundError:
            pass
        data = bytes(make_id())
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, path)
        return data
    t0 = time.monotonic()
    while True:
        try:
            with open(path, "rb") as f:
                data = f.read()
            if data:
                return data
        except FileNotFoundError:
            pass
        if time.monotonic() - t0 > timeout:
            raise TimeoutError(f"rank {rank}: no communicator id at {path} after {timeout:.0f} s")
        time.sleep(0.01)


def cleanup_id(key: str, directory: Optional[str] = None) -> None:
    path = os.path.join(directory or tempfile.gettempdir(), f"dx_comm_{key}.id")
    try:
        os.remove(path)
    except FileNotFoundError:
        pass


class Comm:
    """An RCCL communicator owned by libdx (dx_comm_* in include/dx.h)."""

    def __init__(self, rank: int, world: int, device: int, key: Optional[str] = None):
        L = _lib.load()
        self.rank, self.world, self.device = int(rank), int(world), int(device)
        self.key = key or job_key()

        def make_id() -> bytes:
            buf = ctypes.create_string_buffer(_lib.COMM_ID_BYTES)
            _lib.check(L.dx_comm_unique_id(buf))
            return buf.raw

        uid = exchange_id(self.rank, self.key, make_id)
        self.ptr = L.dx_comm_init(uid, self.world, self.rank, self.device)
        if not self.ptr:
            raise _lib.DxError(f"dx_comm_init failed: {L.dx_last_error().decode()}")
        self.barrier()  # every rank holds the id now
        if self.rank == 0:
            cleanup_id(self.key)

    @classmethod
    def from_env(cls, device: Optional[int] = None) -> "Comm":
        check_single_node()
        rank = int(os.environ.get("RANK", "0"))
        world = int(os.environ.get("WORLD_SIZE", "1"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        return cls(rank, world, local if device is None else device)

    def barrier(self) -> None:
        _lib.check(_lib.load().dx_comm_barrier(self.ptr))

    def max(self, value: float) -> float:
        """Max over ranks of a host scalar (blocking)."""
        v = ctypes.c_double(float(value))
        _lib.check(_lib.load().dx_comm_allreduce_max(self.ptr, ctypes.byref(v)))
        return v.value

    def close(self) -> None:
        if getattr(self, "ptr", None) and _lib._lib is not None:
            _lib._lib.dx_comm_destroy(self.ptr)
        self.ptr = None

    def __del__(self):
        self.close()


class OutputCollator:
    """The gathered [W * n, obs_dim + 3] float32 buffer of a sharded job, in device
    memory on this rank's GPU; `gather()` enqueues dx_allgather_obs on the env's
    stream (no host synchronisation)."""

    def __init__(self, env, comm: Comm):
        self.env, self.comm = env, comm
        self.width = env.obs_dim + 3
        self.rows = comm.world * env.num_envs
        self.nbytes = self.rows * self.width * 4
        self.ptr = _device_alloc(self.nbytes)

    def gather(self) -> int:
        _lib.check(_lib.load().dx_allgather_obs(self.env.ptr, self.comm.ptr, ctypes.c_void_p(self.ptr)))
        return self.ptr

    def read(self):
        """Host copy of the gathered buffer (synchronises the env's stream)."""
        import numpy as np

        from dexterity_amd.manipulation import _copy_d2h

        self.env.physics.sync()
        out = np.empty((self.rows, self.width), dtype=np.float32)
        _copy_d2h(out, self.ptr)
        return out

    def close(self) -> None:
        if getattr(self, "ptr", None):
            _device_free(self.ptr)
        self.ptr = None

    def __del__(self):
        self.close()


def _device_alloc(nbytes: int) -> int:
    from dexterity_amd.manipulation import _hip_runtime

    hip = _hip_runtime()
    p = ctypes.c_void_p()
    rc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes))
    if rc != 0 or not p.value:
        raise _lib.DxError(f"hipMalloc({nbytes}) failed ({rc})")
    return p.value


def _device_free(ptr: int) -> None:
    from dexterity_amd.manipulation import _hip_runtime

    _hip_runtime().hipFree(ctypes.c_void_p(ptr))
