"""Diagnostics for tests/test_gpu_parity.py::test_full_batch_parity: every env of the
bench's state mix whose one-substep result departs from the oracle, classified by whether
an oracle run from a perturbed state reproduces it (fp32 input rounding 6e-8, and fp32
computation-level 1e-6), with the state's acceleration scale; the unexplained ones are
saved to gpurun_out/full_batch_bad.npz for CPU analysis.  -> stdout"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dexterity_amd import _lib, manipulation, physics  # noqa: E402
from oracle import oracle as O  # noqa: E402

n = 4096
env = manipulation.load("reorient", "state_dense", seed=1, num_envs=n)
env.reset()
for step in range(40):
    env.step_random(step)
ph = env.physics
qpos, qvel = ph.qpos, ph.qvel
ws, ctrl = ph.get(_lib.QACC_WARMSTART), ph.get(_lib.CTRL)
xfrc = env.task.gravity_compensation
model = env.model
env.close()
p = physics.BatchedPhysics(model, n)
p.set_xfrc(xfrc)
for f, v in ((_lib.QPOS, qpos), (_lib.QVEL, qvel), (_lib.QACC_WARMSTART, ws), (_lib.CTRL, ctrl)):
    p.set(f, v)
p.debug(True)
p.forward()
a0 = p.debug_get("qacc_smooth")
con = p.debug_get("contact")
gqacc = p.qacc
scale = np.maximum(1.0, np.abs(a0).max(axis=1))
for f, v in ((_lib.QPOS, qpos), (_lib.QVEL, qvel), (_lib.QACC_WARMSTART, ws)):
    p.set(f, v)
p.debug(False)
p.step(1)
gq, gv = p.qpos, p.qvel
p.close()
om = O.OracleModel(model.blob)
x32 = np.asarray(xfrc, dtype=np.float32).astype(np.float64).ravel()
rc, oq, ov, _ = O.batch_step(om, qpos.astype(np.float64), qvel.astype(np.float64), ctrl.astype(np.float64),
                             ws.astype(np.float64), x32, nsub=1)
eq = np.abs(gq - oq).max(axis=1)
ev = np.abs(gv - ov).max(axis=1) / scale
bad = np.flatnonzero((eq > 1e-6) | (ev > 5e-4))
rng = np.random.RandomState(0)
K = 32


def nearest(e, rel):
    Q = np.tile(qpos[e].astype(np.float64), (K, 1))
    V = np.tile(qvel[e].astype(np.float64), (K, 1))
    Q[1:] *= 1 + rng.standard_normal(Q[1:].shape) * rel
    V[1:] *= 1 + rng.standard_normal(V[1:].shape) * rel
    _, pq, pv, _ = O.batch_step(om, Q, V, np.tile(ctrl[e].astype(np.float64), (K, 1)),
                                np.tile(ws[e].astype(np.float64), (K, 1)), x32, nsub=1)
    a = np.abs(pq - gq[e]).max(axis=1)
    b = np.abs(pv - gv[e]).max(axis=1) / scale[e]
    i = int(np.argmin(a + 1e-3 * b))
    return a[i], b[i], np.abs(pq - pq[0]).max()


def excess(e):
    """scale * (f(gpu qacc) - f(oracle qacc)) in the oracle's fp64 problem at state e"""
    d = O.OracleData(om)
    d.qpos[:] = qpos[e]
    d.qvel[:] = qvel[e]
    d.ctrl[:] = ctrl[e]
    d.qacc_warmstart[:] = ws[e]
    d.xfrc_applied[:] = x32
    d.forward()
    oa = d.qacc.copy()
    c0 = d.solver_cost(oa)
    return d.solver_cost(gqacc[e]) - c0, c0, d.niter


tight = np.setdiff1d(np.arange(n), bad)
ex_t = np.array([excess(e)[0] for e in rng.choice(tight, 300, replace=False)])
print(f"cost excess (scaled) of the GPU qacc, tight sample: median {np.median(ex_t):.3g}, 99% {np.quantile(ex_t, 0.99):.3g}, "
      f"max {ex_t.max():.3g}, min {ex_t.min():.3g}")
rows = []
for e in bad:
    a1, b1, s1 = nearest(e, 6e-8)
    a2, b2, s2 = nearest(e, 1e-6)
    x, c0, it = excess(e)
    rows.append((e, eq[e], ev[e], scale[e], a1, b1, s1, a2, b2, s2, x, c0, it))
r = np.array(rows)
ex1 = (r[:, 4] <= 1e-6) & (r[:, 5] <= 5e-4)
ex2 = (r[:, 7] <= 1e-6) & (r[:, 8] <= 5e-4)
print(f"{len(bad)} of {n} outside the tight bound; explained at 6e-8: {ex1.sum()}, at 1e-6 (and not 6e-8): "
      f"{(ex2 & ~ex1).sum()}; unexplained {(~ex1 & ~ex2).sum()}")
print(f"cost excess, explained: median {np.median(r[ex1 | ex2, 10]):.3g} max {r[ex1 | ex2, 10].max():.3g}")
un = r[~ex1 & ~ex2]
order = np.argsort(-un[:, 1])
print("unexplained: env, qpos err, qvel err/scale, scale, nearest(6e-8) q, v, spread, nearest(1e-6) q, v, spread, "
      "cost excess, oracle cost, oracle iterations")
for row in un[order]:
    print(" ".join(f"{x:.3g}" for x in row))
sel = un[:, 0].astype(int)
np.savez(os.path.join(ROOT, "gpurun_out", "full_batch_bad.npz"), env=sel, qpos=qpos[sel], qvel=qvel[sel], ws=ws[sel],
         ctrl=ctrl[sel], gpu_con=con[sel], gpu_qacc=gqacc[sel], gpu_qpos1=gq[sel], gpu_qvel1=gv[sel], eq=eq[sel],
         ev=ev[sel], scale=scale[sel], xfrc=np.asarray(xfrc, dtype=np.float32))
