"""Environment-level GPU tests through the C ABI: the RCCL collation path, the
observation vector against the fp64 restatement, termination paths, and the
reference's closed-loop known-answer tests."""

import os

import numpy as np
import pytest

from dexterity_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def built():
    from dexterity_amd import build

    build.build()


def test_allgather_world1(built):
    """dx_allgather_obs over a one-rank RCCL communicator returns exactly the packed
    [obs | reward | discount | step_type] rows of the env (the in-place gather puts
    rank 0's rows at offset 0)."""
    from dexterity_amd import distributed, manipulation

    env = manipulation.load("reorient", "state_dense", seed=3, num_envs=64, device=0)
    comm = distributed.Comm(0, 1, 0, key=f"gputest_{os.getpid()}")
    col = distributed.OutputCollator(env, comm)
    env.reset()
    for i in range(3):
        env.step(env.sample_actions(i), device_action=True)
        col.gather()
    got = col.read()
    ts = env.timestep()
    obs = np.concatenate([ts.observation[k] for k in ts.observation], axis=1).astype(np.float32)
    assert got.shape == (64, env.obs_dim + 3)
    np.testing.assert_array_equal(got[:, : env.obs_dim], obs)
    np.testing.assert_array_equal(got[:, env.obs_dim], ts.reward.astype(np.float32))
    np.testing.assert_array_equal(got[:, env.obs_dim + 1], ts.discount.astype(np.float32))
    np.testing.assert_array_equal(got[:, env.obs_dim + 2], ts.step_type.astype(np.float32))
    assert comm.max(2.5) == 2.5
    comm.barrier()
    col.close()
    comm.close()
    env.close()
