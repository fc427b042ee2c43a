"""The mid and overflow tiers (dx_step_mid_kernel, dx_step_hi_kernel) against the step
kernel on the bench's state mix: every physics step with a contact forced to the mid tier
(DX_DEFER_AT=0), or through it to the overflow tier (DX_MID_DEFER_AT=0 too, a grid of
DX_HI_GRID workgroups), vs the step kernel alone, from the same 4096 states -- cost per
physics step and results (diagnostics; -> stdout)."""
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


def run(defer_at, grid, nsub, reps=5, mid_defer_at=None):
    for k in ("DX_DEFER_AT", "DX_HI_GRID", "DX_MID_DEFER_AT"):
        os.environ.pop(k, None)
    if defer_at is not None:
        os.environ["DX_DEFER_AT"] = str(defer_at)
        os.environ["DX_HI_GRID"] = str(grid)
    if mid_defer_at is not None:
        os.environ["DX_MID_DEFER_AT"] = str(mid_defer_at)
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
    for name, kw in (("mid tier", dict(defer_at=0, grid=2048)),
                     ("overflow tier", dict(defer_at=0, grid=2048, mid_defer_at=0))):
        (b_q, b_v, b_n, b_h), tb = run(nsub=nsub, **kw)
        diff = (a_q != b_q).any(axis=1) | (a_v != b_v).any(axis=1)
        print(f"nsub {nsub}: step kernel {ta * 1e3:.3f} ms; forced {name} {tb * 1e3:.3f} ms "
              f"(deferred {b_h['contact_deferred']} of {n * nsub} env-substeps); envs not bit-identical {diff.sum()}, "
              f"max |dqpos| {np.abs(a_q - b_q).max():.2e}, max |dqvel| {np.abs(a_v - b_v).max():.2e}, ncon equal "
              f"{(a_n == b_n).mean():.3f}", flush=True)
