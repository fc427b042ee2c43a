"""The overflow tier (dx_step_hi_kernel) against the step kernel on the bench's state mix:
every physics step with a contact forced to the overflow tier (DX_DEFER_AT=0, a grid of
DX_HI_GRID workgroups) vs the step kernel alone, from the same 4096 states -- its cost per
physics step and its results (diagnostics; -> stdout)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dexterity_amd import _lib, manipulation, physics  # noqa: E402

n = 4096
env = manipulation.load("reorient", "state_dense", seed=1, num_envs=n)
env.reset()
for step in range(40):
    env.step_random(step)
ph = env.physics
st = [ph.qpos, ph.qvel, ph.get(_lib.QACC_WARMSTART), ph.get(_lib.CTRL)]
xfrc = env.task.gravity_compensation
model = env.model
env.close()
fields = (_lib.QPOS, _lib.QVEL, _lib.QACC_WARMSTART, _lib.CTRL)


def run(defer_at, grid, nsub, reps=5):
    if defer_at is None:
        os.environ.pop("DX_DEFER_AT", None)
        os.environ.pop("DX_HI_GRID", None)
    else:
        os.environ["DX_DEFER_AT"] = str(defer_at)
        os.environ["DX_HI_GRID"] = str(grid)
    p = physics.BatchedPhysics(model, n)
    p.set_xfrc(xfrc)
    ts = []
    for r in range(reps):
        for f, v in zip(fields, st):
            p.set(f, v)
        p.health_clear()
        p.sync()
        t = time.perf_counter()
        p.step(nsub)
        p.sync()
        ts.append(time.perf_counter() - t)
    out = (p.qpos, p.qvel, p.get(_lib.NCON)[:, 0], p.health())
    p.close()
    return out, min(ts)


for nsub in (1, 5):
    (a_q, a_v, a_n, a_h), ta = run(None, 32, nsub)
    (b_q, b_v, b_n, b_h), tb = run(0, 2048, nsub)
    diff = (a_q != b_q).any(axis=1) | (a_v != b_v).any(axis=1)
    print(f"nsub {nsub}: step kernel {ta * 1e3:.3f} ms; forced overflow tier {tb * 1e3:.3f} ms "
          f"(deferred {b_h['contact_deferred']} of {n * nsub} env-substeps); envs not bit-identical {diff.sum()}, "
          f"max |dqpos| {np.abs(a_q - b_q).max():.2e}, max |dqvel| {np.abs(a_v - b_v).max():.2e}, ncon equal "
          f"{(a_n == b_n).mean():.3f}", flush=True)
