"""Diagnostics for tests/test_gpu_parity.py::test_full_batch_parity: the envs of the bench's
state mix whose one-substep result departs from the oracle -- which dofs, their contact
lists on both sides, constraint counts, solver iterations.  -> stdout"""
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
st = env._read(_lib.OUT_STEP_TYPE, np.int32, 1)[:, 0]
xfrc = env.task.gravity_compensation
model = env.model
cm = env.task.compiled
env.close()
p = physics.BatchedPhysics(model, n)
p.set_xfrc(xfrc)
for f, v in ((_lib.QPOS, qpos), (_lib.QVEL, qvel), (_lib.QACC_WARMSTART, ws), (_lib.CTRL, ctrl)):
    p.set(f, v)
p.debug(True)
p.forward()
a0 = p.debug_get("qacc_smooth")
con = p.debug_get("contact")
cnt = p.debug_get("efc_count")
gqacc = p.qacc
gniter = p.get(_lib.NITER)[:, 0]
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
print(f"{len(bad)} of {n} envs outside the tight bound; step types of those: {np.bincount(st[bad], minlength=3)}"
      f" (all: {np.bincount(st, minlength=3)})")
print("scale of bad envs: p50", np.median(scale[bad]), "max", scale[bad].max(), "; all p50", np.median(scale))
order = bad[np.argsort(-eq[bad])]
kinds = {"contact_set": 0, "same_set": 0}
for e in order[:40]:
    d = O.OracleData(om)
    d.xfrc_applied[:] = x32
    d.qpos[:], d.qvel[:], d.qacc_warmstart[:], d.ctrl[:] = qpos[e], qvel[e], ws[e], ctrl[e]
    d.forward()
    oc = d.contacts()
    gc = con[e, : (con[e, :, 13] != 0).sum()]
    gs = sorted((int(r[13]), int(r[14])) for r in gc)
    os_ = sorted((int(r[13]), int(r[14])) for r in oc)
    same = gs == os_
    kinds["same_set" if same else "contact_set"] += 1
    dq = np.abs(gq[e] - oq[e])
    k = int(np.argmax(dq))
    qa = np.abs(gqacc[e] - d.qacc)
    print(f"env {e}: qpos err {eq[e]:.2e} at dof {k}, qvel err/scale {ev[e]:.2e}, scale {scale[e]:.1f}, "
          f"qacc err max {qa.max():.2e} at {int(np.argmax(qa))}; nefc gpu {cnt[e, 0]} oracle {d.nefc}; "
          f"niter gpu {gniter[e]} oracle {d.niter}; ncon gpu {len(gc)} oracle {len(oc)}; same set {same}")
    if not same:
        print("   gpu only:", sorted(set(gs) - set(os_)), "oracle only:", sorted(set(os_) - set(gs)))
        for r in gc:
            if (int(r[13]), int(r[14])) not in os_:
                print(f"     gpu contact {int(r[13])}-{int(r[14])} dist {r[12]:.3e}")
        for r in oc:
            if (int(r[13]), int(r[14])) not in gs:
                print(f"     oracle contact {int(r[13])}-{int(r[14])} dist {r[12]:.3e}")
    else:
        om_ = {(int(r[13]), int(r[14])): r for r in oc}
        for r in gc:
            o = om_[(int(r[13]), int(r[14]))]
            if abs(r[12] - o[12]) > 2e-5 or np.abs(r[3:6] - o[3:6]).max() > 2e-3 or np.abs(r[0:3] - o[0:3]).max() > 2e-4:
                print(f"     differs {int(r[13])}-{int(r[14])}: dist {r[12]:.3e} vs {o[12]:.3e}, normal err "
                      f"{np.abs(r[3:6] - o[3:6]).max():.2e}, pos err {np.abs(r[0:3] - o[0:3]).max():.2e}")
print(kinds)
sel = order[:64]
np.savez(os.path.join(ROOT, "gpurun_out", "full_batch_bad.npz"), env=sel, qpos=qpos[sel], qvel=qvel[sel], ws=ws[sel],
         ctrl=ctrl[sel], gpu_con=con[sel], gpu_qacc=gqacc[sel], gpu_qpos1=gq[sel], gpu_qvel1=gv[sel], eq=eq[sel],
         ev=ev[sel], xfrc=np.asarray(xfrc, dtype=np.float32))
