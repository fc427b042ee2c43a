"""Quick GPU-vs-oracle probe (development aid; the real checks live in tests/)."""

import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dexterity_amd import _lib, physics  # noqa: E402
from dexterity_amd.mjcf.compiler import CompiledModel  # noqa: E402
from oracle import oracle as O  # noqa: E402

cm = CompiledModel.load("assets/shadow_reorient.npz")
model = physics.Model(cm)
print("sizes nq nv nbody ngeom ncon_max nefc_max", model.nq, model.nv, model.nbody, model.ngeom, model.ncon_max, model.nefc_max)
om = O.OracleModel(model.blob)
xfrc = physics.gravity_compensation(cm, "shadow_hand_e/")

# oracle trajectory: drop cube, 60 steps
od = O.OracleData(om)
od.xfrc_applied[:] = xfrc.ravel()
states = []
for s in range(80):
    od.step()
    if s in (0, 30, 50, 79):
        states.append((od.qpos.copy(), od.qvel.copy(), od.qacc_warmstart.copy()))
B = len(states)
phys = physics.BatchedPhysics(model, B)
phys.set_xfrc(xfrc)
phys.debug(True)
qpos = np.stack([s[0] for s in states]); qvel = np.stack([s[1] for s in states]); ws = np.stack([s[2] for s in states])
phys.set(_lib.QPOS, qpos); phys.set(_lib.QVEL, qvel); phys.set(_lib.QACC_WARMSTART, ws)
phys.forward(); phys.sync()
M = phys.debug_get("M"); a0 = phys.debug_get("qacc_smooth"); con = phys.debug_get("contact"); cnt = phys.debug_get("efc_count")
qacc = phys.qacc
for e in range(B):
    od2 = O.OracleData(om)
    od2.xfrc_applied[:] = xfrc.ravel()
    od2.qpos[:] = qpos[e]; od2.qvel[:] = qvel[e]; od2.qacc_warmstart[:] = ws[e]
    od2.forward()
    Mo = od2.M.reshape(model.nv, model.nv)
    print(f"env{e}: M relerr {np.abs(M[e]-Mo).max()/np.abs(Mo).max():.2e}  qacc_smooth err {np.abs(a0[e]-od2.qacc_smooth).max():.2e} (scale {np.abs(od2.qacc_smooth).max():.2e})")
    print(f"   ncon gpu {int((con[e,:,13]!=0).sum())} oracle {od2.ncon}  nefc gpu {cnt[e]} oracle {od2.nefc}")
    print(f"   qacc err {np.abs(qacc[e]-od2.qacc).max():.3e} scale {np.abs(od2.qacc).max():.3e}")
# stepping
t = time.time()
phys.step(5); phys.sync()
print("step ok", phys.qpos[:, 24:27])
for nenv in (1024, 4096):
    p2 = physics.BatchedPhysics(model, nenv)
    p2.set_xfrc(xfrc)
    p2.set(_lib.QPOS, np.repeat(qpos[2:3], nenv, 0)); p2.set(_lib.QVEL, np.repeat(qvel[2:3], nenv, 0))
    p2.step(5); p2.sync()
    t = time.time()
    for _ in range(10):
        p2.step(5)
    p2.sync()
    dt = (time.time() - t) / 10
    print(f"nenv {nenv}: {dt*1e3:.2f} ms per control step -> {nenv/dt:.0f} env-steps/s; niter {np.bincount(p2.get(_lib.NITER).ravel())}")
