"""Multi-GPU sharding and observation collation.

Environments are independent: rank r of W owns the contiguous env range
`env_shard(B_global, r, W)` on its own GPU and steps it with no data-path
collective.  The only exchange is one all-gather per control step of each rank's
packed `[obs | reward | discount | step_type]` rows (dx_env_pack_outputs), which
over RCCL/xGMI is ~2 MB per rank at 4096 envs.  The same code runs on gloo for the
CPU tests.
"""

from __future__ import annotations

from typing import Tuple


def env_shard(global_envs: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [env0, env0 + n) of rank `rank`; the first `global_envs % world`
    ranks take one extra env."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, extra = divmod(global_envs, world)
    n = base + (1 if rank < extra else 0)
    env0 = rank * base + min(rank, extra)
    return env0, n


def rank_seed(seed: int, rank: int) -> int:
    """Per-rank task seed (env i of the whole job draws from seed + rank stream)."""
    return int(seed) + int(rank)


class OutputCollator:
    """All-gathers equally sized per-rank [n, width] float32 shards into [W*n, width]."""

    def __init__(self, n_per_rank: int, width: int, device):
        import torch
        import torch.distributed as dist

        self.dist = dist
        self.world = dist.get_world_size()
        self.shard = torch.empty((n_per_rank, width), dtype=torch.float32, device=device)
        self.gathered = torch.empty((self.world * n_per_rank, width), dtype=torch.float32, device=device)
        self._use_tensor_api = dist.get_backend() != "gloo"
        if not self._use_tensor_api:
            self._parts = list(self.gathered.chunk(self.world, dim=0))

    def gather(self):
        """Collective over the current contents of `self.shard`; returns `self.gathered`."""
        if self._use_tensor_api:
            self.dist.all_gather_into_tensor(self.gathered, self.shard)
        else:
            parts = [p.clone() for p in self._parts]
            self.dist.all_gather(parts, self.shard)
            for dst, src in zip(self._parts, parts):
                dst.copy_(src)
        return self.gathered


def max_over_ranks(seconds: float, device) -> float:
    """The bench contract's job time: the slowest rank's elapsed seconds."""
    import torch
    import torch.distributed as dist

    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
